// Native MLP executor: plan -> grouped MFMA launches -> hipGraph.
// See executor.h for the step structure.
#include "executor.h"

#include <map>
#include <mutex>

#include <cstdlib>

#include <algorithm>
#include <cstring>

extern "C" hipError_t ea_gemm_grouped(const ea::GroupArgs* ga, int bf16, int cfg, hipStream_t s);
extern "C" int ea_gemm_tile_m(int cfg);
extern "C" int ea_gemm_tile_n(int cfg);
extern "C" void ea_gemm_init();
extern "C" hipError_t ea_gemm_table(const ea::TableArgs* ta, int bf16, int dw, hipStream_t s);
extern "C" hipError_t ea_rowchain(const ea::RcArgs* a, int bf16, int nbw, hipStream_t s);
extern "C" hipError_t ea_apply_update(ea::FlatArgs* a, int bf16, hipStream_t s);
extern "C" hipError_t ea_refresh_shadows(ea::FlatArgs* a, int bf16, hipStream_t s);
extern "C" hipError_t ea_advance(long long* ctr, const int* ntrain, int R, int B, int n, hipStream_t s);
extern "C" hipError_t ea_persist_post_average(unsigned* flags, int nflags, long long* ctr, const int* ntrain, int R,
                                              int B, int n, const unsigned* err, float* P, long long sP, long long np,
                                              float* out, int write_back, double scale, hipStream_t s);
extern "C" hipError_t ea_persist_post(unsigned* flags, int nflags, long long* ctr, const int* ntrain, int R, int B, int n,
                                      const unsigned* err, hipStream_t s);
extern "C" hipError_t ea_persist(const ea::PersistArgs* a, hipStream_t s);
extern "C" hipError_t ea_persist_local(const ea::PersistArgs* a, hipStream_t s);
extern "C" hipError_t ea_persist_xlocal(const ea::PersistArgs* a, hipStream_t s);
extern "C" hipError_t ea_xcc_probe(int nblocks, unsigned* out, hipStream_t s);
extern "C" hipError_t ea_deep_xrank_selftest(const ea::DeepArgs* a, int nsteps, unsigned* bad, int corrupt,
                                             hipStream_t s);
extern "C" int ea_persist_lds_bytes();
extern "C" hipError_t ea_deep(const ea::DeepArgs* a, int local, hipStream_t s);
extern "C" hipError_t ea_xrank_selftest(const ea::PersistArgs* a, int nsteps, unsigned* bad, int corrupt, hipStream_t s);

namespace ea {

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

Executor::Executor(const ExecCfg& cfg) : c_(cfg) {
  if (c_.layers.empty()) throw std::invalid_argument("executor needs at least one Dense layer");
  if (c_.B <= 0 || c_.Bp < c_.B || (c_.Bp % 8) != 0) throw std::invalid_argument("bad batch padding");
  for (auto& l : c_.layers) {
    if (l.Kp % 8 || l.Np % 8 || l.Kp < l.K || l.Np < l.N) throw std::invalid_argument("layer dims must be padded to 8");
  }
  ea_gemm_init();
  build();
  rc_.on = c_.rowchain != 0 && build_rowchain();
  if (c_.rowchain == 1 && !rc_) throw std::invalid_argument("row-chain plan requested but the model is not eligible");
  tl_.on = !rc_ && c_.rowchain != 0 && c_.tail != 0 && build_tail();
  // deep = 2 (tests, A/B): the layer pipeline even where persist.hip's roles are eligible
  dp_.on = c_.persist != 0 && c_.deep == 2 && build_deep();
  pm_.on = !dp_.on && c_.persist != 0 && build_persist();
  if (!dp_.on && !pm_.on) dp_.on = c_.persist != 0 && c_.deep != 0 && build_deep();
  if (c_.persist == 1 && !persistent()) throw std::invalid_argument("persistent plan requested but the model is not eligible");
}

Executor::~Executor() {
  // work still in flight on any stream may use these buffers and graphs (a trainer dropped
  // right after enqueueing): drain the device before freeing anything
  (void)hipDeviceSynchronize();
  destroy_graphs();
  if (d_probs_) (void)hipFree(d_probs_);
  if (d_zp_) (void)hipFree(d_zp_);
  if (d_zw_) (void)hipFree(d_zw_);
  if (d_pws_) (void)hipFree(d_pws_);
  if (d_pflags_) (void)hipFree(d_pflags_);
  if (d_perr_) (void)hipFree(d_perr_);
  if (d_dws_) (void)hipFree(d_dws_);
  if (d_dxg_) (void)hipFree(d_dxg_);
  if (d_dflags_) (void)hipFree(d_dflags_);
}

// Persistent plan (persist.hip): 3 Dense layers, hidden widths 64 or 128, a last layer
// of <= 16 units, fp32, B <= 64, and a grid of at most one workgroup per CU (every
// workgroup must be resident: they wait for each other inside the launch).
// Does the dispatch put blocks b and b + 8 of an n-block grid on one XCD (the XCD-local
// persistent instance's assumption, persist.hip EA_PLOCAL)?  Probed once per device and grid size with
// a tiny kernel reading HW_REG_XCC_ID; the kernel re-checks it at every launch (PERR_PLACE).
static bool xcd_round_robin(int dev, int n) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, bool> seen;
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_pair(dev, n);
  auto it = seen.find(key);
  if (it != seen.end()) return it->second;
  unsigned* d = nullptr;
  bool ok = hipMalloc(&d, sizeof(unsigned) * (size_t)n) == hipSuccess;
  std::vector<unsigned> h(n, 99u);
  ok = ok && ea_xcc_probe(n, d, nullptr) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
       hipMemcpy(h.data(), d, sizeof(unsigned) * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess;
  if (d) (void)hipFree(d);
  // the dispatch deals blocks round-robin over the 8 XCDs, starting wherever the previous
  // dispatch stopped (tools/micro/xcc_map.hip: block 0 on XCD 6 after other launches): the
  // premise is that blocks b and b + 8 share an XCD, and the 8 residues use 8 XCDs
  for (int b = 0; ok && b < n; ++b) ok = h[b] == h[b % 8];
  for (int i = 0; ok && i < 8 && i < n; ++i)
    for (int k = 0; k < i; ++k) ok = ok && h[i] != h[k];
  seen[key] = ok;
  return ok;
}

bool Executor::build_persist() {
  auto no_pm = [&](const char* why) { why_pm_ = why; return false; };
  const int L = (int)c_.layers.size();
  if (L != 3) return no_pm("persist.hip: 3 Dense layers only");
  const LayerCfg &l0 = c_.layers[0], &l1 = c_.layers[1], &l2 = c_.layers[2];
  // hidden widths (64, 64), (128, 128) or (128, 64): the kernel is compiled for those shapes
  if (!((l0.N == 64 && l1.N == 64) || (l0.N == 128 && l1.N == 128) || (l0.N == 128 && l1.N == 64)))
    return no_pm("persist.hip: hidden widths (64, 64), (128, 128) or (128, 64) only");
  if (l1.K != l0.N || l2.K != l1.N || l2.N > PM_MAXC || c_.ldy > 32) return no_pm("persist.hip: a last layer of <= 16 units");
  if (c_.B > PM_ROWS || c_.B < 1) return no_pm("persist.hip: batch <= 64 rows per replica");
  const int nch = cdiv(c_.B, 16);
  if (cdiv(l1.N / 16, nch) > PM_NTU) return no_pm("persist.hip: too few chain workgroups for the layer-1 tiles");
  int dev = 0, ncu = 0;
  check(hipGetDevice(&dev), "hipGetDevice");
  check(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
  if (const char* e = std::getenv("ELEPHAS_AMD_PERSIST_CUS")) ncu = std::min(ncu, std::atoi(e));  // tests: a smaller grid
  // tests only: pretend the GPU has more CUs than it does, so the grid cannot be resident
  // (the kernel's GO-flag wait must fail cleanly and the host fall back)
  if (const char* e = std::getenv("ELEPHAS_AMD_PERSIST_OVERSUBSCRIBE")) ncu = std::max(ncu, std::atoi(e));
  if (c_.persist_cus > 0) ncu = std::min(ncu, c_.persist_cus);  // a share of the GPU (concurrent executors)
  int lds_max = 0;
  check(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev), "hipDeviceGetAttribute");
  if (ea_persist_lds_bytes() > lds_max) return no_pm("persist.hip: LDS");
  const int cap = std::min(ncu / c_.R - nch, PM_MAXWG);
  if (cap < 1) return no_pm("persist.hip: not enough CUs for the replicas' clusters");
  // V2 (persist.hip l0_role_v2 / dw_role_v2): plain SGD, ReLU hidden layers, independent
  // replicas -- the step's critical path runs through the chain workgroups only
  // (the chain's Gram correction carries layer 0's bias update -- its ones column -- so a
  // bias-free first layer keeps the V1 roles)
  const bool v2 = c_.persist_v2 != 0 && !c_.persist_sync && c_.op.opt == OPT_SGD && c_.op.mom == 0.f &&
                  l0.act == ACT_RELU && l1.act == ACT_RELU && l0.has_bias;
  const int nd = v2 ? cdiv(l1.N / 16, PM_NTU) : 0;
  // bf16 (mixed_bfloat16): the V2 roles only (bf16-rounded operands, bf16 shard and images)
  if (c_.bf16 && !v2) return no_pm("persist.hip: mixed_bfloat16 needs the V2 roles (plain SGD, ReLU, layer-0 bias)");
  // layer-0 tiles: the cheapest (kc0, cw) whose tile count fits.  V1: cost ~ the tile's
  // MFMA work (FWD reduction padded to 64) + the partials every chain workgroup sums.
  // V2: the L0 work is off the critical path; the chain's slab loads (nk0 Pold + Gram
  // slabs) are not -- fewest k-chunks first, then the smaller tile
  int best_kc = 0, best_cw = 0;
  long long best_cost = -1;
  for (int cw : {16, 32, 64}) {
    if (l0.N % cw) continue;
    const int nc0 = l0.N / cw;
    if (v2 ? (cw == 16 || nc0 > 4) : cw == 64) continue;
    for (int kc = 16; kc <= PM_MAXH; kc += 16) {
      const int nk0 = cdiv(l0.K, kc);
      if (nk0 > RC_MAXSPLIT) continue;
      if (v2) {
        if (kc > 112) continue;   // three X chunks of kc + 1 columns in LDS (persist.hip L0V2_LDS)
        if (nk0 * nc0 + nd > cap) continue;
        const long long cost = 100000LL * nk0 + (long long)kc * cw;
        if (best_cost < 0 || cost < best_cost) { best_cost = cost; best_kc = kc; best_cw = cw; }
        continue;
      }
      if (nk0 * nc0 > cap || (kc / 16) * (cw / 16) > 16) continue;
      const long long cost = (long long)(cdiv(std::min(kc, l0.K), 64) * 64 + kc) * cw + 512LL * nk0;
      if (best_cost < 0 || cost < best_cost) { best_cost = cost; best_kc = kc; best_cw = cw; }
    }
  }
  if (best_cost < 0) return no_pm("persist.hip: no layer-0 tiling fits the CUs");
  PersistArgs& a = pm_.args;
  std::memset(&a, 0, sizeof(a));
  a.R = c_.R; a.B = c_.B;
  a.K0 = l0.K; a.H0 = l0.N; a.H1 = l1.N; a.C = l2.N;
  a.kc0 = best_kc; a.cw = best_cw; a.nc0 = l0.N / best_cw; a.nk0 = cdiv(l0.K, best_kc);
  // V2: one weight-gradient workgroup per layer-1 column tile when the CUs allow (halves
  // their MFMA chain vs two tiles each: the W1 / W2 hand-off is on the step's critical path)
  const int nd_use = (v2 && cdiv(l0.K, best_kc) * (l0.N / best_cw) + l1.N / 16 <= cap) ? l1.N / 16 : nd;
  a.nch = nch; a.v2 = v2 ? 1 : 0; a.nd = nd_use;
  // V2 Gram slabs on the weight-gradient workgroups (off the layer-0 tiles' loop, which is
  // on the step's critical path) when every k-chunk fits their LDS (<= 112 columns, even
  // for the bf16 pairs); otherwise on the layer-0 tiles
  const char* gl0 = std::getenv("ELEPHAS_AMD_PERSIST_GRAM_L0");   // A/B: keep them on the layer-0 tiles
  if (v2 && !(gl0 && std::atoi(gl0) != 0)) {
    const int gk = (cdiv(l0.K, nd_use) + 1) & ~1;
    if (gk <= 112) { a.gk = gk; a.ng = cdiv(l0.K, gk); }
  }
  a.wgs = a.nk0 * a.nc0 + nch + nd_use;
  a.sync = c_.persist_sync ? 1 : 0;
  // XCD-local instances (persist.hip EA_PLOCAL), where the dispatch deals blocks round-robin
  // over the XCDs: fit -- block b serves replica b % R, so with R a multiple of 8 every
  // replica's cluster sits on one XCD (intra-replica hand-offs in its L2); per-step sync of 8
  // replicas on the V1 roles -- the 8 copies of each workgroup on one XCD (the exchange in
  // its L2).  The PS hook's in-launch exchange keeps the write-through instance.
  pm_.local = 0;
  if (c_.persist_local != 0 && xcd_round_robin(dev, c_.R * a.wgs)) {
    if (!a.sync && c_.R % 8 == 0) pm_.local = 1;
    else if (a.sync && !v2 && c_.R == 8 && a.wgs % 8 == 0) pm_.local = 2;
  }
  const char* xrs = std::getenv("ELEPHAS_AMD_XCHG_RS");   // A/B: reduce-scatter exchange of the replicas
  a.xchg_rs = (xrs && std::atoi(xrs) != 0) ? 1 : 0;
  a.bf16 = c_.bf16 ? 1 : 0;
  const char* pim = std::getenv("ELEPHAS_AMD_PERSIST_IMAGES");   // A/B: V2 epilogue writes the images too
  a.imgs = (!v2 || (pim && std::atoi(pim) != 0)) ? 1 : 0;
  a.act0 = l0.act; a.act1 = l1.act; a.act2 = l2.act;
  a.rate0 = l0.rate; a.rate1 = l1.rate;
  a.bias0 = l0.has_bias; a.bias1 = l1.has_bias; a.bias2 = l2.has_bias;
  a.p_off0 = l0.p_off; a.p_off1 = l1.p_off; a.p_off2 = l2.p_off;
  a.X = reinterpret_cast<const float*>(c_.X); a.sX = c_.sX; a.ldx = c_.ldx;
  a.Y = reinterpret_cast<const float*>(c_.Y); a.sY = c_.sY; a.ldy = c_.ldy;
  a.perm = reinterpret_cast<const int*>(c_.perm); a.sPerm = c_.sPerm;
  a.ntrain = reinterpret_cast<const int*>(c_.ntrain);
  a.P = reinterpret_cast<float*>(c_.P); a.sP = c_.sP;
  a.S = reinterpret_cast<float*>(c_.S); a.sS = c_.sS;
  a.op = c_.op;
  a.Wsh = reinterpret_cast<float*>(c_.Wsh); a.sWsh = c_.sWsh; a.wsh_par = c_.wsh_par;
  a.WTsh = reinterpret_cast<float*>(c_.WTsh); a.sWTsh = c_.sWTsh; a.wtsh_par = c_.wtsh_par;
  for (int l = 0; l < 3; ++l) {
    a.wsh_off[l] = c_.layers[l].wsh_off; a.wtsh_off[l] = c_.layers[l].wtsh_off;
    a.Np[l] = c_.layers[l].Np; a.Kp[l] = c_.layers[l].Kp;
  }
  a.loss = c_.loss; a.nmet = c_.nmet;
  for (int i = 0; i < 4; ++i) a.met[i] = c_.met[i];
  a.acc = reinterpret_cast<double*>(c_.acc); a.acc_stride = c_.acc_stride;
  a.ctr = reinterpret_cast<long long*>(c_.ctr);
  a.seed = c_.seed;
  // exchange workspace per replica (floats; every region 64-float aligned)
  long long off = 0;
  auto take = [&](long long n) { const long long o = off; off += (n + 63) / 64 * 64; return o; };
  // V2 double-buffers the partials, the Gram slabs and dZ_0 by step parity
  const int npar = v2 ? 2 : 1;
  a.part_par = v2 ? (long long)a.nk0 * PM_ROWS * a.H0 : 0;
  a.o_part = take(npar * (long long)a.nk0 * PM_ROWS * a.H0);
  const int nslab = std::max(a.nk0, a.ng);
  a.g_par = v2 ? (long long)nslab * PM_ROWS * PM_ROWS : 0;
  a.o_g = v2 ? take(3LL * nslab * PM_ROWS * PM_ROWS) : 0;   // three Gram slabs (step % 3)
  a.dz0_par = v2 ? (long long)PM_ROWS * a.H0 : 0;
  a.o_dz0 = take(npar * (long long)PM_ROWS * a.H0);
  a.o_a0 = take((long long)PM_ROWS * a.H0);
  a.o_a1 = take((long long)PM_ROWS * a.H1);
  a.o_dz1 = take((long long)PM_ROWS * a.H1);
  a.o_dz2 = take((long long)PM_ROWS * 16);
  a.o_w1 = take((long long)a.H0 * a.H1);
  a.o_w2 = take((long long)a.H1 * 16);
  a.o_b1 = take(a.H1);
  a.o_b2 = take(16);
  a.o_xg = a.sync ? take(2LL * a.wgs * PM_XSLOT) : 0;
  a.o_xt = a.sync ? take(2LL * a.wgs * PM_XSLOT) : 0;   // used with the rank exchange
  a.ws_stride = off;
  const size_t ws_bytes = sizeof(float) * (size_t)off * c_.R;
  check(hipMalloc(&d_pws_, ws_bytes), "hipMalloc(persistent workspace)");
  check(hipMemset(d_pws_, 0, ws_bytes), "hipMemset(persistent workspace)");
  pm_.flag_bytes = sizeof(unsigned) * (size_t)c_.R * PMF_N * PM_MAXWG;
  check(hipMalloc(&d_pflags_, pm_.flag_bytes), "hipMalloc(persistent flags)");
  check(hipMemset(d_pflags_, 0, pm_.flag_bytes), "hipMemset(persistent flags)");
  check(hipMalloc(&d_perr_, 256), "hipMalloc(persistent error word)");
  check(hipMemset(d_perr_, 0, 256), "hipMemset(persistent error word)");
  a.ws = d_pws_;
  a.flags = d_pflags_;
  a.err = d_perr_;
  a.timeout = std::max<long long>(1, c_.persist_timeout_ms) * 100000LL;  // s_memrealtime: 100 MHz
  // the zeroed flags and error word must be in memory before the first launch, which
  // goes to a caller's (non-blocking) stream that does not order after hipMemset's
  check(hipDeviceSynchronize(), "hipDeviceSynchronize(persistent plan setup)");
  return true;
}

// Persistent layer pipeline (deep.hip): 2..DP_MAXL Dense layers, hidden widths <= 1024, a
// last layer of <= DP_MAXC units, B <= DP_ROWS, fp32, independent replicas (fit
// granularity).  nw = the widest hidden layer's 16-column tiles workgroups per replica,
// at most one workgroup per CU (every one resident: they wait for each other).
bool Executor::build_deep() {
  auto no_dp = [&](const char* why) { why_dp_ = why; return false; };
  const int L = (int)c_.layers.size();
  if (L < 2 || L > DP_MAXL) return no_dp("layer pipeline: 2..5 Dense layers");
  if (c_.bf16) return no_dp("layer pipeline: fp32 only");
  if (c_.B < 1 || c_.B > DP_ROWS) return no_dp("layer pipeline: batch <= 128 rows per replica");
  if (c_.ldy > 32) return no_dp("layer pipeline: label rows of <= 32 columns");
  if ((c_.ldx % 8) != 0) return no_dp("layer pipeline: a feature stride that is a multiple of 8");
  const LayerCfg& lastc = c_.layers[L - 1];
  if (lastc.N > DP_MAXC) return no_dp("layer pipeline: a last layer of <= 32 units");
  auto r16 = [](int n) { return (n + 15) / 16 * 16; };
  int nw = 0;
  for (int l = 0; l < L - 1; ++l) {
    const int n16 = r16(c_.layers[l].N);
    if (n16 > 1024) return no_dp("layer pipeline: hidden widths <= 1024");
    nw = std::max(nw, n16 / 16);
    if (l > 0 && c_.layers[l].K != c_.layers[l - 1].N) return no_dp("layer pipeline: a plain Dense chain");
  }
  if (lastc.K != c_.layers[L - 2].N || c_.layers[0].K > c_.ldx) return no_dp("layer pipeline: a plain Dense chain");
  if (nw > DP_MAXWG) return no_dp("layer pipeline: too many column tiles");
  int dev = 0, ncu = 0, lds_max = 0;
  check(hipGetDevice(&dev), "hipGetDevice");
  check(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
  check(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev), "hipDeviceGetAttribute");
  if (const char* e = std::getenv("ELEPHAS_AMD_PERSIST_OVERSUBSCRIBE")) ncu = std::max(ncu, std::atoi(e));
  if (c_.persist_cus > 0) ncu = std::min(ncu, c_.persist_cus);
  if (c_.R * nw > ncu) return no_dp("layer pipeline: replicas x widest-layer tiles > CUs");
  DeepArgs& a = dp_.args;
  std::memset(&a, 0, sizeof(a));
  a.R = c_.R; a.B = c_.B; a.L = L; a.nw = nw;
  int rt = 1;
  while (rt * 16 < c_.B) rt *= 2;
  a.RT = rt; a.KS = 8 / rt; a.Bp = 16 * rt;
  // layers, LDS layout (floats; every region a multiple of 4), workspace layout (floats,
  // 64-float aligned regions)
  int lds = 0;
  long long ws = 0;
  auto take = [&](long long n) { const long long o = ws; ws += (n + 63) / 64 * 64; return o; };
  for (int l = 0; l < L; ++l) {
    const LayerCfg& ly = c_.layers[l];
    DeepLayer& d = a.ly[l];
    d.K = ly.K; d.N = ly.N; d.N16 = r16(ly.N); d.T = d.N16 / 16;
    d.Kx = l == 0 ? (int)c_.ldx : a.ly[l - 1].N16;
    d.act = ly.act; d.has_bias = ly.has_bias; d.rate = ly.rate; d.p_off = ly.p_off;
  }
  a.ly[0].l_w = lds; lds += 16 * (a.ly[0].Kx + 4);
  for (int l = 1; l < L; ++l) { a.ly[l].l_w = lds; lds += 16 * (a.ly[l].N16 + 4); }
  for (int l = 0; l < L - 1; ++l) { a.ly[l].l_b = lds; lds += 16; }
  a.ly[L - 1].l_b = lds; lds += 32;
  for (int l = 0; l < L - 1; ++l) { a.ly[l].l_at = lds; lds += 16 * (a.Bp + 4); }
  // the dZ_0^T stripe doubles as bw_phase's second DW-partial buffer ([4][64][4] floats)
  a.l_dz0 = lds; lds += std::max(16 * (a.Bp + 4), 4 * 64 * 4);
  a.l_red = lds; lds += 2048;
  int stage = DP_ROWS * (DP_CW + 4) + 1024;                          // backward dZ chunk + DW partials
  stage = std::max(stage, 8 * 2 * 256 + 16 * 36 + 16 * 32 + 16);     // tail tiles
  stage = std::max(stage, a.Bp * (a.ly[L - 1].N16 + 4));             // dZ_{L-1} of the last layer's DW
  for (int l = 1; l < L - 1; ++l) stage = std::max(stage, 16 * (a.ly[l].Kx + 4));   // W^T stripes
  stage = std::max(stage, 16 * a.ly[L - 1].Kx);                       // the tail's dZ_{L-2} rows
  a.l_stage = lds; lds += stage;
  lds += 2 * DP_ROWS;                                                 // batch rows of two steps (ints, last)
  a.lds_floats = lds;
  if ((long long)lds * 4 + 1024 > lds_max) return no_dp("layer pipeline: the owned tiles exceed the LDS");   // + static LDS
  for (int l = 0; l < L - 1; ++l) {
    a.ly[l].o_a = take((long long)a.Bp * a.ly[l].N16);
    a.ly[l].o_dz = take((long long)a.Bp * a.ly[l].N16);
  }
  a.ly[L - 1].o_dz = take((long long)a.Bp * a.ly[L - 1].N16);
  a.o_g = take((long long)a.Bp * a.ly[L - 2].N16);
  for (int l = 1; l < L; ++l) a.ly[l].o_wt = take((long long)a.ly[l].N16 * a.ly[l].Kx);
  a.ly[L - 1].o_w = take((long long)a.ly[L - 1].Kx * a.ly[L - 1].N16);
  a.o_bl = take(a.ly[L - 1].N16);
  a.X = reinterpret_cast<const float*>(c_.X); a.sX = c_.sX; a.ldx = c_.ldx;
  a.Y = reinterpret_cast<const float*>(c_.Y); a.sY = c_.sY; a.ldy = c_.ldy;
  a.perm = reinterpret_cast<const int*>(c_.perm); a.sPerm = c_.sPerm;
  a.ntrain = reinterpret_cast<const int*>(c_.ntrain);
  a.P = reinterpret_cast<float*>(c_.P); a.sP = c_.sP;
  const bool sgd0 = c_.op.opt == OPT_SGD && c_.op.mom == 0.f;
  a.S = sgd0 ? nullptr : reinterpret_cast<float*>(c_.S); a.sS = c_.sS;
  a.op = c_.op;
  a.loss = c_.loss; a.nmet = c_.nmet;
  for (int i = 0; i < 4; ++i) a.met[i] = c_.met[i];
  a.acc = reinterpret_cast<double*>(c_.acc); a.acc_stride = c_.acc_stride;
  a.ctr = reinterpret_cast<long long*>(c_.ctr);
  a.seed = c_.seed;
  a.ws_stride = ws;
  // the gradient-tile layout of the exchange buffer (per-step synchronous replicas, and the
  // parameter-server hook -- set_param_server allocates it then)
  a.sync = c_.persist_sync ? 1 : 0;
  {
    int xt = 16 * a.ly[0].Kx;
    a.x_b0 = xt; xt += 16;
    for (int l = 1; l < L; ++l) {
      a.x_w[l] = xt; xt += 16 * a.ly[l].N16;
      a.x_b[l] = xt; xt += 32;
    }
    a.XT = (xt + 63) / 64 * 64;
  }
  if (a.sync) {
    const size_t xb = sizeof(float) * (size_t)a.XT * (size_t)(c_.R + 1) * (size_t)nw;
    check(hipMalloc(&d_dxg_, xb), "hipMalloc(layer pipeline exchange buffer)");
    a.xg = d_dxg_;
  }
  // the XCD-local instances (deep_l*_local.hip): fit granularity, R a multiple of 8
  dp_.local = c_.persist_local != 0 && !a.sync && c_.R % 8 == 0 && xcd_round_robin(dev, c_.R * nw);
  const size_t ws_bytes = sizeof(float) * (size_t)ws * c_.R;
  check(hipMalloc(&d_dws_, ws_bytes), "hipMalloc(layer pipeline workspace)");
  check(hipMemset(d_dws_, 0, ws_bytes), "hipMemset(layer pipeline workspace)");
  dp_.flag_bytes = sizeof(unsigned) * (size_t)c_.R * 4 * DP_MAXWG;
  check(hipMalloc(&d_dflags_, dp_.flag_bytes), "hipMalloc(layer pipeline flags)");
  check(hipMemset(d_dflags_, 0, dp_.flag_bytes), "hipMemset(layer pipeline flags)");
  if (!d_perr_) {
    check(hipMalloc(&d_perr_, 256), "hipMalloc(persistent error word)");
    check(hipMemset(d_perr_, 0, 256), "hipMemset(persistent error word)");
  }
  a.ws = d_dws_;
  a.flags = d_dflags_;
  a.err = d_perr_;
  a.timeout = std::max<long long>(1, c_.persist_timeout_ms) * 100000LL;   // s_memrealtime: 100 MHz
  // the zeroed flags and error word are in memory before the first launch (a caller's
  // non-blocking stream does not order after hipMemset's)
  check(hipDeviceSynchronize(), "hipDeviceSynchronize(layer pipeline setup)");
  return true;
}

std::vector<int> Executor::deep_geometry() const {
  if (!dp_.on) return {};
  const DeepArgs& a = dp_.args;
  return {a.nw, a.R * a.nw, a.RT, a.KS, a.lds_floats * 4, a.XT};
}

std::vector<int> Executor::persist_geometry() const {
  if (dp_.on) return {0, 0, 0, 0, 0, dp_.args.nw, dp_.args.R * dp_.args.nw};
  if (!pm_.on) return {};
  const PersistArgs& a = pm_.args;
  return {a.nk0, a.nc0, a.kc0, a.cw, a.nch, a.wgs, a.R * a.wgs};
}

bool Executor::set_param_server(const PsArgs& ps, int mode) {
  if (dp_.on) {   // the layer pipeline: gradient tiles through xg, push / pull per step (deep_impl.h exchange)
    if (dp_.args.sync || ps.nchunks <= 0 || dp_.args.nw > PEER_MAX_BLOCKS) return mode == 0;
    DeepArgs& a = dp_.args;
    if (!d_dxg_) {
      const size_t xb = sizeof(float) * (size_t)a.XT * (size_t)(c_.R + 1) * (size_t)a.nw;
      check(hipMalloc(&d_dxg_, xb), "hipMalloc(layer pipeline exchange buffer)");
      check(hipDeviceSynchronize(), "hipDeviceSynchronize(layer pipeline exchange buffer)");
    }
    a.xg = d_dxg_;
    a.ps = ps;
    a.ps_mode = mode;
    if (mode) dp_.local = false;   // the hook runs on the write-through instances
    return true;
  }
  if (!pm_.on || pm_.args.v2 || pm_.args.sync) return mode == 0;
  pm_.args.ps = ps;
  pm_.args.ps_mode = mode;
  return true;
}

bool Executor::set_rank_exchange(const std::vector<char*>& bases, int world, int rank, unsigned tag0,
                                 double timeout_s) {
  if (dp_.on) {   // the layer pipeline (deep_impl.h exchange + deep_xrank_wait)
    DeepArgs& a = dp_.args;
    if (!a.sync || world > PEER_MAX_RANKS || (int)bases.size() != world || rank < 0 || rank >= world ||
        a.R * a.nw > 2 * PEER_MAX_BLOCKS)
      return world <= 1;
    for (int k = 0; k < PEER_MAX_RANKS; ++k) a.xr_base[k] = k < world ? bases[k] : nullptr;
    a.xr_world = world;
    a.xr_rank = rank;
    a.xr_timeout = (long long)(std::max(1.0, timeout_s) * 1e8);   // s_memrealtime: 100 MHz
    a.timeout = std::max(a.timeout, a.xr_timeout);
    dp_.xr_steps = tag0;
    return true;
  }
  if (!pm_.on || !pm_.args.sync || world > PEER_MAX_RANKS || (int)bases.size() != world || rank < 0 ||
      rank >= world || pm_.args.wgs > PEER_MAX_BLOCKS)
    return world <= 1;
  PersistArgs& a = pm_.args;
  // the exchange-local instance's replica exchange was only validated on one rank (the
  // 2-process tests cannot hold 8 replicas per rank on one GPU): across ranks, write-through
  if (world > 1 && pm_.local == 2) pm_.local = 0;
  for (int k = 0; k < PEER_MAX_RANKS; ++k) a.xr_base[k] = k < world ? bases[k] : nullptr;
  a.xr_world = world;
  a.xr_rank = rank;
  a.xr_timeout = (long long)(std::max(1.0, timeout_s) * 1e8);   // s_memrealtime: 100 MHz
  // every in-launch wait may now sit behind another rank (startup skew of seconds): the
  // rank exchange's patience for all of them (residency was checked on the host)
  a.timeout = std::max(a.timeout, a.xr_timeout);
  pm_.xr_steps = tag0;   // a rebuilt executor continues the trainer's tag sequence
  return true;
}

// Numeric self-test of the attached rank exchange (persist.hip xrank_selftest_kernel):
// nsteps exchanges of known integer tiles on every owning workgroup, checked against the
// exact rank sums.  Collective (every rank runs it, the tags advance on all of them).
// Returns {workgroup-steps with a wrong element, workgroups that timed out}.
std::vector<unsigned> Executor::rank_exchange_selftest(int nsteps, int corrupt) {
  const bool deep = dp_.on && dp_.args.xr_world > 1;
  if (!deep && (!pm_.on || pm_.args.xr_world <= 1)) return {0u, 0u};
  if (nsteps <= 0) return {0u, 0u};
  unsigned* d = nullptr;
  check(hipMalloc(&d, sizeof(unsigned)), "hipMalloc(self-test word)");
  check(hipMemset(d, 0, sizeof(unsigned)), "hipMemset(self-test word)");
  check(hipDeviceSynchronize(), "hipDeviceSynchronize(self-test setup)");
  hipError_t e;
  if (deep) {
    DeepArgs a = dp_.args;
    a.xr_tag0 = dp_.xr_steps;
    dp_.xr_steps += (unsigned)nsteps;
    e = ea_deep_xrank_selftest(&a, nsteps, d, corrupt, nullptr);
  } else {
    PersistArgs a = pm_.args;
    a.xr_tag0 = pm_.xr_steps;
    pm_.xr_steps += (unsigned)nsteps;
    e = ea_xrank_selftest(&a, nsteps, d, corrupt, nullptr);
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  unsigned v = 0;
  if (e == hipSuccess) e = hipMemcpy(&v, d, sizeof(v), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  check(e, "rank-exchange self-test");
  if (persist_error() == PERR_XRANK) persist_clear_error();   // the timeout is reported in the result
  return {v & 0xFFFFu, v >> 16};
}

std::vector<int> Executor::persist_variant() const {
  if (dp_.on) return {3, 0, dp_.args.sync, dp_.local && !dp_.args.ps_mode ? 1 : 0};
  if (!pm_.on) return {};
  return {pm_.args.v2 ? 2 : 1, pm_.args.nd, pm_.args.sync, pm_.local};
}

unsigned Executor::persist_error() const {
  if (!d_perr_) return 0;
  unsigned v = 0;
  check(hipMemcpy(&v, d_perr_, sizeof(v), hipMemcpyDeviceToHost), "hipMemcpy(persistent error word)");
  return v;
}

void Executor::persist_clear_error() {
  if (d_perr_) {
    check(hipMemset(d_perr_, 0, 256), "hipMemset(persistent error word)");
    check(hipDeviceSynchronize(), "hipDeviceSynchronize(persistent error word)");
  }
}

void Executor::run_chunk(hipStream_t s, int nsteps) const {
  if (dp_.on) {   // one persistent launch + the post node (flag clear, counter advance)
    DeepArgs a = dp_.args;
    a.nsteps = nsteps;
    if (a.xr_world > 1) {   // the rank exchange's flag tags continue over launches
      a.xr_tag0 = dp_.xr_steps;
      dp_.xr_steps += (unsigned)nsteps;
    }
    check(ea_deep(&a, dp_.local && !a.sync && !a.ps_mode ? 1 : 0, s), "persistent layer pipeline kernel");
    chunk_post(d_dflags_, dp_.flag_bytes, nsteps, s);
    return;
  }
  if (pm_.on) {
    // the flags are zero at launch (setup, then the post node of every chunk: tags
    // restart at 1), and one post node clears them again and advances the counters
    // (instead of a flag memset ahead of the launch plus the advance node after it).
    // Measured, not kept: the kernel's last workgroup doing both (async 'batch' +15 %,
    // but the step loop ran 2-3 % slower: profiles/persist_exit_ab_r3.txt)
    PersistArgs a = pm_.args;
    a.nsteps = nsteps;
    if (pm_.avg) {   // train_chunk_avg: this launch ends with the fused replica averaging
      a.avg_end = 1;
      a.avg_p = pm_.avg->avg_p;
      a.avg_n = pm_.avg->avg_n;
      a.avg_scale = pm_.avg->avg_scale;
      a.avg_out = pm_.avg->avg_out;
    }
    if (a.xr_world > 1) {   // the rank exchange's flag tags continue over launches
      a.xr_tag0 = pm_.xr_steps;
      pm_.xr_steps += (unsigned)nsteps;
    }
    check(pm_.local == 1 ? ea_persist_local(&a, s) : pm_.local == 2 ? ea_persist_xlocal(&a, s) : ea_persist(&a, s),
          "persistent step kernel");
    chunk_post(d_pflags_, pm_.flag_bytes, nsteps, s);
    return;
  }
  for (int i = 0; i < nsteps; ++i) run_step(s, i);
}

// the post node of a persistent chunk: flag clear + counter advance, and (train_chunk_avg
// mode 2) the replica averaging in the same launch
void Executor::chunk_post(unsigned* flags, size_t flag_bytes, int nsteps, hipStream_t s) const {
  const int nflags = (int)(flag_bytes / sizeof(unsigned));
  long long* ctr = reinterpret_cast<long long*>(c_.ctr);
  const int* ntrain = reinterpret_cast<const int*>(c_.ntrain);
  if (post_avg_) {
    check(ea_persist_post_average(flags, nflags, ctr, ntrain, c_.R, c_.B, nsteps, d_perr_,
                                  reinterpret_cast<float*>(c_.P), c_.sP, c_.nparams, post_avg_->out,
                                  post_avg_->write_p, post_avg_->scale, s),
          "persistent chunk post + replica average");
    return;
  }
  check(ea_persist_post(flags, nflags, ctr, ntrain, c_.R, c_.B, nsteps, d_perr_, s), "persistent chunk post");
}

// Row-chain plan (rowchain.hip): 2 <= L <= RC_MAXL Dense layers, every layer but
// the last at most RC_MAXW wide, a last layer of at most 32 units (its loss runs
// on whole rows inside one workgroup).
bool Executor::build_rowchain() {
  const int L = (int)c_.layers.size();
  if (L < 2 || L > RC_MAXL || L > TABLE_MAX) return false;
  int wmax = 0;
  for (int l = 0; l < L - 1; ++l) wmax = std::max(wmax, c_.layers[l].N);
  if (wmax > RC_MAXW || c_.layers[L - 1].N > 32 || c_.ldy > 32) return false;
  if (fwd_.empty() || fwd_[0].ga.nprob != 2 || fwd_[0].ga.p[0].kind != PK_FWD || fwd_[0].ga.p[1].kind != PK_GATHER_T)
    return false;
  if ((int)bwd_.size() != L) return false;
  const LayerCfg& l0 = c_.layers[0];
  // split-K slabs of layer 0: chunks of >= ~112 reduction elements (K = 784 -> 7)
  int ns = c_.rc_split > 0 ? c_.rc_split : cdiv(l0.Kp, 112);
  ns = std::max(1, std::min(ns, RC_MAXSPLIT));
  const int kchunk = cdiv(cdiv(l0.Kp, ns), 8) * 8;
  ns = cdiv(l0.Kp, kchunk);
  rc_.nsplitk = ns;
  rc_.nbw = wmax <= 128 ? 2 : 4;
  const long long slab = (long long)c_.B * l0.Np;  // rows padded to 8: 16-byte slab reads
  check(hipMalloc(&d_zp_, sizeof(float) * (size_t)c_.R * ns * slab), "hipMalloc(row-chain slabs)");
  check(hipMemset(d_zp_, 0, sizeof(float) * (size_t)c_.R * ns * slab), "hipMemset(row-chain slabs)");

  auto table = [&](TableArgs& ta, Prob* host, int n, Prob* dev, int cfg) { make_table(ta, host, n, dev, cfg); };
  check(hipMalloc(&d_probs_, sizeof(Prob) * 3 * TABLE_MAX), "hipMalloc(problem tables)");

  // A: layer-0 product as split-K slabs + the X^T gather (from the grouped FWD_0 launch)
  Prob pa[2] = {fwd_[0].ga.p[0], fwd_[0].ga.p[1]};
  Prob& z = pa[0];
  z.kind = PK_PARTIAL;
  z.tiles_k = ns;
  z.kchunk = kchunk;
  z.D = d_zp_;
  z.ldd = l0.Np;
  z.sD = ns * slab;
  z.sPart = slab;
  z.Z = nullptr;
  z.DT = nullptr;
  table(rc_.ta_fwd, pa, 2, d_probs_, 0);

  // C: DW of every layer (the grouped plan's DW problems), update and gradient forms
  Prob pu[TABLE_MAX], pg[TABLE_MAX];
  for (int l = 0; l < L; ++l) {
    pu[l] = bwd_[L - 1 - l].ga.p[0];  // bwd_ runs from the last layer down
    if (pu[l].kind != PK_DW_UPDATE) return false;
    pg[l] = pu[l];
    pg[l].kind = PK_DW_GRAD;
    // (layer 0's update already skips its reader-less row-major image, build(): the
    // split-K slab launch and the evaluation executor read W^T, the row chain reads W
    // and W^T of layers >= 1 only)
  }
  table(rc_.ta_dw, pu, L, d_probs_ + TABLE_MAX, 3);
  table(rc_.ta_grad, pg, L, d_probs_ + 2 * TABLE_MAX, 3);

  // B: the row chain
  RcArgs& a = rc_.rc;
  std::memset(&a, 0, sizeof(a));
  a.L = L; a.R = c_.R; a.B = c_.B; a.Bp = c_.Bp;
  a.nsplitk = ns;
  a.Zp = d_zp_; a.sZp = ns * slab; a.sZpk = slab;
  for (int l = 0; l < L; ++l) {
    const LayerCfg& ly = c_.layers[l];
    RcLayer& q = a.ly[l];
    q.K = ly.K; q.N = ly.N; q.Kp = ly.Kp; q.Np = ly.Np;
    q.act = ly.act; q.has_bias = ly.has_bias; q.rate = ly.rate;
    q.p_off = ly.p_off; q.wsh_off = ly.wsh_off; q.wtsh_off = ly.wtsh_off;
    q.DT = reinterpret_cast<void*>(ly.DT);
    q.dZT = reinterpret_cast<void*>(ly.dZT);
  }
  a.Y = reinterpret_cast<const float*>(c_.Y); a.sY = c_.sY; a.ldy = c_.ldy;
  a.perm = reinterpret_cast<const int*>(c_.perm); a.sPerm = c_.sPerm;
  a.ntrain = reinterpret_cast<const int*>(c_.ntrain);
  a.P = reinterpret_cast<const float*>(c_.P); a.sP = c_.sP;
  a.Wsh = reinterpret_cast<const void*>(c_.Wsh); a.sWsh = c_.sWsh; a.wsh_par = c_.wsh_par;
  a.WTsh = reinterpret_cast<const void*>(c_.WTsh); a.sWTsh = c_.sWTsh; a.wtsh_par = c_.wtsh_par;
  a.loss = c_.loss; a.nmet = c_.nmet;
  for (int i = 0; i < 4; ++i) a.met[i] = c_.met[i];
  a.acc = reinterpret_cast<double*>(c_.acc); a.acc_stride = c_.acc_stride;
  a.ctr = reinterpret_cast<long long*>(c_.ctr);
  a.seed = c_.seed;
  return true;
}

// tile geometry of the table launches: 64x32 (cfg 0: layer-0 / tail slabs), 64x64
// (cfg 3: weight gradients); problem i owns tiles [begin[i], begin[i+1]) per replica
void Executor::make_table(TableArgs& ta, Prob* host, int n, Prob* dev, int cfg) const {
  const int bm = ea_gemm_tile_m(cfg), bn = ea_gemm_tile_n(cfg);
  std::memset(&ta, 0, sizeof(ta));
  int begin = 0;
  for (int i = 0; i < n; ++i) {
    Prob& p = host[i];
    if (p.kind == PK_GATHER_T) {
      p.tiles_m = cdiv(p.B, 64);
      p.tiles_n = cdiv(p.K, 64);
    } else {
      p.tiles_m = cdiv(p.M, bm);
      p.tiles_n = cdiv(p.N, bn);
    }
    if (p.kind != PK_PARTIAL) p.tiles_k = 1;
    p.block_begin = 0;
    ta.begin[i] = begin;
    begin += p.tiles_m * p.tiles_n * std::max(1, p.tiles_k);
  }
  ta.probs = dev;
  ta.nprob = n;
  ta.R = c_.R;
  ta.total_blocks = begin;
  ta.ctr = reinterpret_cast<long long*>(c_.ctr);
  ta.seed = c_.seed;
  check(hipMemcpy(dev, host, sizeof(Prob) * n, hipMemcpyHostToDevice), "hipMemcpy(problem table)");
}

// Tail-chain plan: the row chain (rowchain.hip, L = 2) over the last two layers of a
// deeper stack whose layer L-2 is at most RC_TAILW wide and whose last layer has at
// most 32 units (Otto: 512 -> 9). The chain starts from the pre-activations z_{L-2}
// the grouped FWD_{L-2} launch stored (activation and dropout recomputed in-row), and
// replaces the loss launch (FWD_{L-1}: 2 workgroups per replica at B = 128) and the
// last layer's input-gradient launch; DW_{L-1} joins a backward launch with a free slot.
bool Executor::build_tail() {
  const int L = (int)c_.layers.size();
  if (L < 3 || (int)fwd_.size() != L || (int)bwd_.size() < L) return false;
  const LayerCfg& la = c_.layers[L - 2];
  const LayerCfg& lb = c_.layers[L - 1];
  if (la.N > RC_TAILW || lb.N > 32 || c_.ldy > 32) return false;
  if (fwd_[L - 2].ga.p[0].kind != PK_FWD || !fwd_[L - 2].ga.p[0].Z) return false;
  if (fwd_[L - 1].ga.nprob != 1 || fwd_[L - 1].ga.p[0].kind != PK_FWD_LOSS) return false;
  // bwd_: [DW_{L-1} (+ DX_{L-1})] or [DW_{L-1}] [DX_{L-1}], then layer L-2's launch(es)
  const Prob dw_last = bwd_[0].ga.p[0];
  if (dw_last.kind != PK_DW_UPDATE) return false;
  const int i = (bwd_[0].ga.nprob == 2) ? 1 : 2;  // skip them (DX_{L-1} runs in the chain)
  if (i == 2 && (bwd_[1].ga.nprob != 1 || bwd_[1].ga.p[0].kind != PK_DX)) return false;
  if (i >= (int)bwd_.size() || bwd_[i].ga.p[0].kind != PK_DW_UPDATE) return false;
  tl_.nbw = la.N <= 128 ? 2 : la.N <= 256 ? 4 : 8;
  tl_.pre.assign(fwd_.begin(), fwd_.begin() + (L - 1));

  // DW_{L-1} needs only the chain's outputs: it rides in the first backward launch
  // with a free problem slot (Otto: DW_{L-2}'s), else it gets its own launch
  tl_.post.assign(bwd_.begin() + i, bwd_.end());
  bool placed = false;
  for (auto& La : tl_.post) {
    if (La.ga.nprob == 1) {
      La.ga.p[1] = dw_last;
      La.ga.nprob = 2;
      finalize(La);
      placed = true;
      break;
    }
  }
  if (!placed) {
    Launch La;
    std::memset(&La, 0, sizeof(La));
    La.ga.p[0] = dw_last;
    La.ga.nprob = 1;
    La.cfg = bwd_[0].cfg >= 100 ? (bwd_[0].cfg - 100) / 10 : bwd_[0].cfg;
    finalize(La);
    tl_.post.insert(tl_.post.begin(), La);
  }

  RcArgs& a = tl_.rc;
  std::memset(&a, 0, sizeof(a));
  a.L = 2; a.R = c_.R; a.B = c_.B; a.Bp = c_.Bp;
  a.nsplitk = 0;
  for (int l = 0; l < 2; ++l) {
    const LayerCfg& ly = c_.layers[L - 2 + l];
    RcLayer& q = a.ly[l];
    q.K = ly.K; q.N = ly.N; q.Kp = ly.Kp; q.Np = ly.Np;
    q.act = ly.act; q.has_bias = ly.has_bias; q.rate = ly.rate;
    q.p_off = ly.p_off; q.wsh_off = ly.wsh_off; q.wtsh_off = ly.wtsh_off;
    q.DT = reinterpret_cast<void*>(ly.DT);
    q.dZT = reinterpret_cast<void*>(ly.dZT);
  }
  a.Y = reinterpret_cast<const float*>(c_.Y); a.sY = c_.sY; a.ldy = c_.ldy;
  a.perm = reinterpret_cast<const int*>(c_.perm); a.sPerm = c_.sPerm;
  a.ntrain = reinterpret_cast<const int*>(c_.ntrain);
  a.P = reinterpret_cast<const float*>(c_.P); a.sP = c_.sP;
  a.Wsh = reinterpret_cast<const void*>(c_.Wsh); a.sWsh = c_.sWsh; a.wsh_par = c_.wsh_par;
  a.WTsh = reinterpret_cast<const void*>(c_.WTsh); a.sWTsh = c_.sWTsh; a.wtsh_par = c_.wtsh_par;
  a.loss = c_.loss; a.nmet = c_.nmet;
  for (int k = 0; k < 4; ++k) a.met[k] = c_.met[k];
  a.acc = reinterpret_cast<double*>(c_.acc); a.acc_stride = c_.acc_stride;
  a.ctr = reinterpret_cast<long long*>(c_.ctr);
  a.seed = c_.seed;
  a.l0 = L - 2;
  a.Zsrc = reinterpret_cast<const float*>(la.Z);
  a.ldzs = la.N;
  a.dZ0 = reinterpret_cast<void*>(la.dZ);
  a.ldz0 = la.Np;
  return true;
}

void Executor::run_tail(hipStream_t s, int step_off) const {
  run(tl_.pre, s, step_off);
  RcArgs a = tl_.rc;
  a.step_off = step_off;
  check(ea_rowchain(&a, c_.bf16, tl_.nbw, s), "tail chain");
  run(tl_.post, s, step_off);
}

void Executor::run_rowchain(hipStream_t s, int step_off, bool grad) const {
  TableArgs ta = rc_.ta_fwd;
  ta.step_off = step_off;
  check(ea_gemm_table(&ta, c_.bf16, 0, s), "row-chain layer-0 slabs");
  RcArgs a = rc_.rc;
  a.step_off = step_off;
  check(ea_rowchain(&a, c_.bf16, rc_.nbw, s), "row chain");
  TableArgs tw = grad ? rc_.ta_grad : rc_.ta_dw;
  tw.step_off = step_off;
  check(ea_gemm_table(&tw, c_.bf16, 1, s), "row-chain weight gradients");
}

void Executor::run_step(hipStream_t s, int step_off) const {
  if (rc_) {
    run_rowchain(s, step_off, false);
  } else if (tl_.on) {
    run_tail(s, step_off);
  } else {
    run(fwd_, s, step_off);
    run(bwd_, s, step_off);
  }
}

// A new dropout seed for every launch of every plan (a refit that reuses this executor:
// the reference starts every fit with a fresh worker model).  Captured graphs hold the
// old arguments and are dropped; buffers, flags and plans stay (no allocation, no sync).
void Executor::set_seed(unsigned long long seed) {
  c_.seed = seed;
  for (auto* v : {&fwd_, &bwd_, &tl_.pre, &tl_.post})
    for (auto& L : *v) L.ga.seed = seed;
  rc_.ta_fwd.seed = rc_.ta_dw.seed = rc_.ta_grad.seed = seed;
  rc_.rc.seed = seed;
  tl_.rc.seed = seed;
  pm_.args.seed = seed;
  dp_.args.seed = seed;
  destroy_graphs();
}

void Executor::destroy_graphs() {
  if (graphs_.empty()) return;
  (void)hipDeviceSynchronize();   // an instantiated graph may still be executing
  for (auto& g : graphs_) {
    if (g.second) (void)hipGraphExecDestroy(g.second);
    if (g.first) (void)hipGraphDestroy(g.first);
  }
  graphs_.clear();
}

// split-K factor for the unfused (wide-output) last layer: THR tiles only, each slab
// at least 8 k-tiles deep, up to LOSS_MAX_SPLIT slabs, until ~2 workgroups per CU
int Executor::split_last(int cfg, long long N, long long K) const {
  if (cfg != 1 && cfg != 2) return 1;
  const char* e = std::getenv("ELEPHAS_AMD_SPLIT_LAST");
  if (e && e[0] == '0') return 1;
  const long long tiles = (long long)c_.R * cdiv((int)c_.B, 128) * cdiv((int)N, ea_gemm_tile_n(cfg));
  int ks = 1;
  while (ks < LOSS_MAX_SPLIT && tiles * ks < 512 && K / (2 * ks) >= 512) ks *= 2;
  return ks;
}

static bool big_dw_off() {
  const char* e = std::getenv("ELEPHAS_AMD_BIG_DW");
  return e && e[0] == '0';
}

int Executor::pick_cfg(long long M, long long N, long long K) const {
  if (c_.force_cfg >= 0) return (c_.force_cfg == 4 && !c_.bf16) ? 1 : c_.force_cfg;
  // 256x256 ping-pong tiles (bf16): by default where the launch holds at least two rounds
  // of them (Wide MLP, 8 workers: 8 x 272 DW tiles, 8 x 64 FWD tiles -- 2.44 M vs 2.19 M
  // samples/s on the THR tiles; 1 worker, one round: 1.48 M vs 1.81 M, profiles/sweep_r5.jsonl);
  // big = 1 forces them wherever they give every CU a workgroup, 0 never
  const long long big_tiles = (long long)c_.R * cdiv((int)M, 256) * cdiv((int)N, 256);
  if (c_.bf16 && c_.big != 0 && M >= 1024 && N >= 1024 && K >= 512 && big_tiles >= (c_.big > 0 ? 240 : 512))
    return 4;
  if (M >= 256 && N >= c_.thr_min_n && K >= c_.thr_min_k) {
    // 128x128 tiles while they give every CU at least two workgroups (256 CUs),
    // else 128x64 tiles (twice the workgroups; measured on MI355X, profiles/)
    const long long tiles = (long long)c_.R * cdiv((int)M, 128) * cdiv((int)N, 128);
    return tiles >= 512 ? 1 : 2;
  }
  return 0;
}

Prob Executor::base_prob() const {
  Prob p;
  std::memset(&p, 0, sizeof(p));
  p.R = c_.R;
  p.B = c_.B;
  p.perm = reinterpret_cast<const int*>(c_.perm);
  p.sPerm = c_.sPerm;
  p.ntrain = reinterpret_cast<const int*>(c_.ntrain);
  p.vstart = reinterpret_cast<const int*>(c_.vstart);
  p.vcount = reinterpret_cast<const int*>(c_.vcount);
  p.ones_row = -1;
  p.op = c_.op;
  p.loss = c_.loss;
  p.nmet = c_.nmet;
  for (int i = 0; i < 4; ++i) p.met[i] = c_.met[i];
  p.acc_stride = c_.acc_stride;
  return p;
}

void Executor::finalize(Launch& L) const {
  int begin = 0;
  for (int i = 0; i < L.ga.nprob; ++i) {
    // a dual launch (cfg 100 + 10 a + b) tiles problem 0 with config a, problem 1 with b
    const int pc = L.cfg >= 100 ? (i == 0 ? (L.cfg - 100) / 10 : L.cfg % 10) : L.cfg;
    const int bm = ea_gemm_tile_m(pc), bn = ea_gemm_tile_n(pc);
    Prob& p = L.ga.p[i];
    // the epilogues' transposed stores move 8 consecutive elements at a time
    if (p.DT && (p.lddt % 8 || p.sDT % 8))
      throw std::invalid_argument("transposed output needs 8-element aligned rows");
    if (p.WTsh && (p.ldwtsh % 8 || p.sWTsh % 8 || p.wtsh_par % 8))
      throw std::invalid_argument("W^T image needs 8-element aligned rows");
    if (p.kind == PK_GATHER_T) {
      p.tiles_m = cdiv(p.B, 64);
      p.tiles_n = cdiv(p.K, 64);
    } else if (p.kind == PK_LOSS_ROWS) {
      p.tiles_m = cdiv(p.M, LOSS_RPB);  // rows per workgroup of the loss rows kernel
      p.tiles_n = 1;
    } else {
      p.tiles_m = cdiv(p.M, bm);
      p.tiles_n = cdiv(p.N, bn);
    }
    p.block_begin = begin;
    // tiles per replica: grid (R, tiles); split-K problems have tiles_k slabs each
    begin += p.tiles_m * p.tiles_n * (p.kind == PK_PARTIAL ? std::max(1, p.tiles_k) : 1);
  }
  // A weight-gradient + input-gradient pair: the problem with the deeper reduction (the
  // longer tiles -- Wide DX, K = 4096, against DW's K = batch) takes the first block
  // range, so its tiles are dispatched first and the short ones fill in around them
  // instead of trailing at the end of the launch
  if (L.ga.nprob == 2) {
    Prob &p0 = L.ga.p[0], &p1 = L.ga.p[1];
    auto gemm_kind = [](int k) { return k == PK_DW_UPDATE || k == PK_DW_GRAD || k == PK_DX; };
    if (gemm_kind(p0.kind) && gemm_kind(p1.kind) && p1.K > p0.K && !c_.no_reorder) {
      p1.block_begin = 0;
      p0.block_begin = p1.tiles_m * p1.tiles_n;
    }
  }
  L.ga.R = c_.R;
  L.ga.total_blocks = begin;
  L.ga.ctr = reinterpret_cast<long long*>(c_.ctr);
  L.ga.seed = c_.seed;
}

std::vector<Executor::Launch> Executor::build_forward(bool eval, long long chunk, const EvalSource* src) const {
  const size_t esz = c_.bf16 ? 2 : 4;
  const int L = (int)c_.layers.size();
  std::vector<Launch> out;
  for (int l = 0; l < L; ++l) {
    const LayerCfg& ly = c_.layers[l];
    const bool last = l == L - 1;
    Prob p = base_prob();
    p.eval_mode = eval ? 1 : 0;
    p.chunk = chunk;
    if (eval) {
      p.vstart = reinterpret_cast<const int*>(src->vstart);
      p.vcount = reinterpret_cast<const int*>(src->vcount);
    }
    p.M = c_.B;
    p.N = ly.N;
    p.K = ly.Kp;
    if (l == 0) {
      p.A = reinterpret_cast<const void*>(eval ? src->X : c_.X);
      p.lda = eval ? src->ldx : c_.ldx;
      p.sA = eval ? src->sX : c_.sX;
      p.a_gather = 1;
    } else {
      const LayerCfg& pv = c_.layers[l - 1];
      p.A = reinterpret_cast<const void*>(pv.D);
      p.lda = pv.Np;
      p.sA = (long long)c_.B * pv.Np;
    }
    p.BT = reinterpret_cast<const void*>(c_.WTsh + ly.wtsh_off * esz);
    p.ldb = ly.Kp;
    p.sB = c_.sWTsh;
    p.bt_shadow = 1;
    p.bt_par = c_.wtsh_par;
    p.bias = ly.has_bias ? reinterpret_cast<const float*>(c_.P) + ly.p_off + (long long)ly.K * ly.N : nullptr;
    p.sBias = c_.sP;
    p.layer = l;
    p.act = ly.act;
    p.rate = ly.rate;
    int cfg = pick_cfg(c_.B, ly.N, ly.Kp);
    if (cfg == 4 && last) cfg = 1;  // the big tile has no loss / split-K epilogue
    Launch La;
    std::memset(&La, 0, sizeof(La));
    La.cfg = cfg;
    if (!last) {
      p.kind = PK_FWD;
      p.Z = reinterpret_cast<float*>(ly.Z);
      p.ldz = ly.N;
      p.sZ = (long long)c_.B * ly.N;
      p.D = reinterpret_cast<void*>(ly.D);
      p.ldd = ly.Np;
      p.sD = (long long)c_.B * ly.Np;
      if (!eval) {
        p.DT = reinterpret_cast<void*>(ly.DT);
        p.lddt = c_.Bp;
        p.sDT = (long long)ly.N * c_.Bp;
      }
      La.ga.p[0] = p;
      La.ga.nprob = 1;
    } else {
      // loss / prediction plumbing
      p.Y = reinterpret_cast<const float*>(eval ? src->Y : c_.Y);
      p.ldy = eval ? src->ldy : c_.ldy;
      p.sY = eval ? src->sY : c_.sY;
      p.acc = reinterpret_cast<double*>(eval ? src->acc : c_.acc);
      if (eval) {
        p.pred = reinterpret_cast<float*>(src->pred);
        p.ldp = src->ldp;
        p.sPred = src->sPred;
      }
      const bool fused = ly.N <= ea_gemm_tile_n(cfg);
      if (fused) {
        p.kind = PK_FWD_LOSS;
        if (!eval) {
          p.D = reinterpret_cast<void*>(ly.dZ);
          p.ldd = ly.Np;
          p.sD = (long long)c_.B * ly.Np;
          p.DT = reinterpret_cast<void*>(ly.dZT);
          p.lddt = c_.Bp;
          p.sDT = (long long)ly.N * c_.Bp;
        }
        La.ga.p[0] = p;
        La.ga.nprob = 1;
      } else {
        Prob g = p;
        g.kind = PK_FWD;
        g.act = ACT_LINEAR;
        g.rate = 0.f;
        g.Z = reinterpret_cast<float*>(ly.Z);
        g.ldz = ly.N;
        g.sZ = (long long)c_.B * ly.N;
        g.D = nullptr;
        g.DT = nullptr;
        g.acc = nullptr;
        g.pred = nullptr;
        // A wide last layer (1024 x 1000 x 4096) gives a 128x64 grid of only 128
        // workgroups: split its reduction into ks slabs (fp32, executor-owned) until
        // every CU holds ~2 workgroups; the loss rows kernel sums the slabs + bias
        const int ks = split_last(cfg, ly.N, ly.Kp);
        if (ks > 1) {
          const long long slab = (long long)c_.B * ly.N;
          if (!d_zw_) check(hipMalloc(&d_zw_, sizeof(float) * (size_t)c_.R * ks * slab), "hipMalloc(logit slabs)");
          g.kind = PK_PARTIAL;
          g.tiles_k = ks;
          g.kchunk = cdiv(cdiv(ly.Kp, ks), 64) * 64;
          g.D = d_zw_;
          g.ldd = ly.N;
          g.sD = ks * slab;
          g.sPart = slab;
          g.Z = nullptr;
          g.bias = nullptr;
        }
        La.ga.p[0] = g;
        La.ga.nprob = 1;
        finalize(La);
        out.push_back(La);
        // wave-per-row loss over the logits
        Prob q = p;
        q.kind = PK_LOSS_ROWS;
        q.Z = reinterpret_cast<float*>(ly.Z);
        q.ldz = ly.N;
        q.sZ = (long long)c_.B * ly.N;
        q.tiles_k = 1;
        if (ks > 1) {
          q.Z = d_zw_;
          q.sZ = ks * (long long)c_.B * ly.N;
          q.tiles_k = ks;
          q.sPart = (long long)c_.B * ly.N;
        }
        if (!eval) {
          q.D = reinterpret_cast<void*>(ly.dZ);
          q.ldd = ly.Np;
          q.sD = (long long)c_.B * ly.Np;
          q.DT = reinterpret_cast<void*>(ly.dZT);
          q.lddt = c_.Bp;
          q.sDT = (long long)ly.N * c_.Bp;
        }
        std::memset(&La, 0, sizeof(La));
        La.cfg = cfg;
        La.ga.p[0] = q;
        La.ga.nprob = 1;
      }
    }
    if (l == 0 && !eval && L > 0) {
      // X^T of the batch for the layer-0 weight gradient, in the same launch
      Prob t = base_prob();
      t.kind = PK_GATHER_T;
      t.A = reinterpret_cast<const void*>(c_.X);
      t.lda = c_.ldx;
      t.sA = c_.sX;
      t.K = ly.Kp;
      t.DT = reinterpret_cast<void*>(c_.XT);
      t.lddt = c_.Bp;
      t.sDT = (long long)ly.Kp * c_.Bp;
      if (La.ga.nprob == 1 && La.ga.p[0].kind != PK_LOSS_ROWS && La.cfg != 4) {
        La.ga.p[1] = t;
        La.ga.nprob = 2;
      } else {
        Launch Lt;
        std::memset(&Lt, 0, sizeof(Lt));
        Lt.cfg = 0;
        Lt.ga.p[0] = t;
        Lt.ga.nprob = 1;
        finalize(Lt);
        out.push_back(Lt);
      }
    }
    finalize(La);
    out.push_back(La);
  }
  return out;
}

void Executor::build() {
  fwd_ = build_forward(false, 0, nullptr);
  bwd_.clear();
  const size_t esz = c_.bf16 ? 2 : 4;
  const int L = (int)c_.layers.size();
  for (int l = L - 1; l >= 0; --l) {
    const LayerCfg& ly = c_.layers[l];
    Prob w = base_prob();
    w.kind = PK_DW_UPDATE;
    if (l == 0) {
      w.A = reinterpret_cast<const void*>(c_.XT);
      w.sA = (long long)ly.Kp * c_.Bp;
    } else {
      const LayerCfg& pv = c_.layers[l - 1];
      w.A = reinterpret_cast<const void*>(pv.DT);
      w.sA = (long long)pv.N * c_.Bp;
    }
    w.lda = c_.Bp;
    w.M = ly.K + (ly.has_bias ? 1 : 0);
    w.ones_row = ly.has_bias ? ly.K : -1;
    w.N = ly.N;
    w.K = c_.Bp;
    w.BT = reinterpret_cast<const void*>(ly.dZT);
    w.ldb = c_.Bp;
    w.sB = (long long)ly.N * c_.Bp;
    w.P = reinterpret_cast<float*>(c_.P);
    w.sP = c_.sP;
    w.p_off = ly.p_off;
    w.S = reinterpret_cast<float*>(c_.S);
    w.sS = c_.sS;
    w.G = reinterpret_cast<float*>(c_.G);
    w.sG = c_.sG;
    // layer 0 has no input gradient: its row-major image (the DX operand) has no reader
    // (the FWD and evaluation launches read W^T), so its update skips that store
    w.Wsh = (l == 0 && c_.rc_lean) ? nullptr : reinterpret_cast<void*>(c_.Wsh + ly.wsh_off * esz);
    w.sWsh = c_.sWsh;
    w.ldwsh = ly.Np;
    w.wsh_par = c_.wsh_par;
    w.WTsh = reinterpret_cast<void*>(c_.WTsh + ly.wtsh_off * esz);
    w.sWTsh = c_.sWTsh;
    w.ldwtsh = ly.Kp;
    w.wtsh_par = c_.wtsh_par;
    Launch La;
    std::memset(&La, 0, sizeof(La));
    long long work = (long long)w.M * w.N * w.K;
    La.ga.p[0] = w;
    La.ga.nprob = 1;
    int cm = (int)w.M, cn = w.N, ck = w.K;
    if (l >= 1) {
      const LayerCfg& pv = c_.layers[l - 1];
      Prob x = base_prob();
      x.kind = PK_DX;
      x.A = reinterpret_cast<const void*>(ly.dZ);
      x.lda = ly.Np;
      x.sA = (long long)c_.B * ly.Np;
      x.BT = reinterpret_cast<const void*>(c_.Wsh + ly.wsh_off * esz);
      x.ldb = ly.Np;
      x.sB = c_.sWsh;
      x.bt_shadow = 1;
      x.bt_par = c_.wsh_par;
      x.M = c_.B;
      x.N = ly.K;
      x.K = ly.Np;
      x.act = pv.act;
      x.rate = pv.rate;
      x.layer = l - 1;
      x.Z = reinterpret_cast<float*>(pv.Z);
      x.ldz = pv.N;
      x.sZ = (long long)c_.B * pv.N;
      x.D = reinterpret_cast<void*>(pv.dZ);
      x.ldd = pv.Np;
      x.sD = (long long)c_.B * pv.Np;
      x.DT = reinterpret_cast<void*>(pv.dZT);
      x.lddt = c_.Bp;
      x.sDT = (long long)pv.N * c_.Bp;
      int cw = pick_cfg(w.M, w.N, w.K);
      const int cx = pick_cfg(x.M, x.N, x.K);
      // A/B: the weight-gradient products on the 128x128 tiles (two workgroups per CU, so
      // one's update epilogue -- bandwidth-bound when every CU reaches it at once -- overlaps
      // the other's main loop) while the input gradients keep the 256x256 tile
      if (cw == 4 && big_dw_off()) cw = 1;
      // the shared launch's tile is the larger product's; when that tile leaves the
      // launch short of two workgroups per CU while the two products prefer different
      // tiles, each gets its own launch (Otto 512x512 layers: DW 513x512x128 on 128x64
      // tiles = 320 workgroups but DX 128x512x512 on them only 64, each reducing K = 512
      // alone -- 58 us; on its own 64x32 split-K tile DX is 256 workgroups)
      const long long wwork = (long long)w.M * w.N * w.K, xwork = (long long)x.M * x.N * x.K;
      const int cs = pick_cfg(xwork > wwork ? x.M : w.M, xwork > wwork ? x.N : w.N, xwork > wwork ? x.K : w.K);
      auto tiles = [&](const Prob& p, int c) {
        return (long long)c_.R * cdiv(p.M, ea_gemm_tile_m(c)) * cdiv(p.N, ea_gemm_tile_n(c));
      };
      const bool underfilled = cw != cx && tiles(w, cs) + tiles(x, cs) < 512;
      if (underfilled && cw == 2 && cx == 0 && c_.dual) {
        // the two products in ONE launch, each on its own tile (gemm_dual)
        La.ga.p[1] = x;
        La.ga.nprob = 2;
        La.cfg = 100 + 10 * cw + cx;
        finalize(La);
        bwd_.push_back(La);
        continue;
      }
      if ((cw == 4) != (cx == 4) || underfilled) {
        // one of the two products fills the chip with 256x256 tiles, the other
        // would leave most CUs idle on them: two launches, each on its own tile
        La.cfg = cw;
        finalize(La);
        bwd_.push_back(La);
        std::memset(&La, 0, sizeof(La));
        La.ga.p[0] = x;
        La.ga.nprob = 1;
        La.cfg = cx;
        finalize(La);
        bwd_.push_back(La);
        continue;
      }
      La.ga.p[1] = x;
      La.ga.nprob = 2;
      long long xw = (long long)x.M * x.N * x.K;
      if (xw > work) { cm = x.M; cn = x.N; ck = x.K; }
    }
    La.cfg = pick_cfg(cm, cn, ck);
    if (La.ga.nprob == 1 && La.cfg == 4 && big_dw_off()) La.cfg = 1;   // layer 0: DW alone
    finalize(La);
    bwd_.push_back(La);
  }
}

void Executor::run(const std::vector<Launch>& ls, hipStream_t s, int step_off) const {
  for (const auto& L : ls) {
    GroupArgs ga = L.ga;
    ga.step_off = step_off;
    check(ea_gemm_grouped(&ga, c_.bf16, L.cfg, s), "gemm_grouped");
  }
}

void Executor::advance(int nsteps, hipStream_t s) const {
  check(ea_advance(reinterpret_cast<long long*>(c_.ctr), reinterpret_cast<const int*>(c_.ntrain), c_.R, c_.B, nsteps, s),
        "advance");
}

void Executor::train_launch(int idx, hipStream_t s) {
  // one launch of the active step plan, step_off 0, no counter advance
  if (rc_) {
    if (idx == 0) check(ea_gemm_table(&rc_.ta_fwd, c_.bf16, 0, s), "train_launch");
    else if (idx == 1) check(ea_rowchain(&rc_.rc, c_.bf16, rc_.nbw, s), "train_launch");
    else check(ea_gemm_table(&rc_.ta_dw, c_.bf16, 1, s), "train_launch");
    return;
  }
  if (tl_.on) {
    const int np = (int)tl_.pre.size();
    if (idx < np) {
      check(ea_gemm_grouped(&tl_.pre[idx].ga, c_.bf16, tl_.pre[idx].cfg, s), "train_launch");
    } else if (idx == np) {
      check(ea_rowchain(&tl_.rc, c_.bf16, tl_.nbw, s), "train_launch");
    } else {
      const Launch& L = tl_.post[idx - np - 1];
      check(ea_gemm_grouped(&L.ga, c_.bf16, L.cfg, s), "train_launch");
    }
    return;
  }
  const int nf = (int)fwd_.size();
  const Launch& L = idx < nf ? fwd_[idx] : bwd_[idx - nf];
  check(ea_gemm_grouped(&L.ga, c_.bf16, L.cfg, s), "train_launch");
}

int Executor::grad_launch_layer(int idx) const {
  const int nf = (int)fwd_.size();
  if (idx < nf) return -1;
  return (int)c_.layers.size() - 1 - (idx - nf);
}

void Executor::grad_launch(int idx, hipStream_t s) {
  const int nf = (int)fwd_.size();
  if (idx < 0 || idx >= grad_launches()) throw std::out_of_range("grad_launch index");
  Launch L = idx < nf ? fwd_[idx] : bwd_[idx - nf];
  for (int i = 0; i < L.ga.nprob; ++i)
    if (L.ga.p[i].kind == PK_DW_UPDATE) L.ga.p[i].kind = PK_DW_GRAD;
  L.ga.step_off = 0;
  check(ea_gemm_grouped(&L.ga, c_.bf16, L.cfg, s), "grad_launch");
}

void Executor::set_stamps(uintptr_t buf) {
  long long* p = reinterpret_cast<long long*>(buf);
  for (auto* v : {&fwd_, &bwd_})
    for (auto& L : *v) L.ga.stamps = p;
  rc_.ta_fwd.stamps = rc_.ta_dw.stamps = rc_.ta_grad.stamps = p;
  rc_.rc.stamps = p;
  pm_.args.stamps = p;
  dp_.args.stamps = p;
  for (auto* v : {&tl_.pre, &tl_.post})
    for (auto& L : *v) L.ga.stamps = p;
  tl_.rc.stamps = p;
}

std::vector<int> Executor::launch_blocks() const {
  std::vector<int> v;
  if (rc_) {
    v.push_back(c_.R * rc_.ta_fwd.total_blocks);
    v.push_back(c_.R * cdiv(c_.B, RC_ROWS));
    v.push_back(c_.R * rc_.ta_dw.total_blocks);
    return v;
  }
  if (tl_.on) {
    for (auto& L : tl_.pre) v.push_back(c_.R * L.ga.total_blocks);
    v.push_back(c_.R * cdiv(c_.B, RC_ROWS));
    for (auto& L : tl_.post) v.push_back(c_.R * L.ga.total_blocks);
    return v;
  }
  for (auto& L : fwd_) v.push_back(c_.R * L.ga.total_blocks);
  for (auto& L : bwd_) v.push_back(c_.R * L.ga.total_blocks);
  return v;
}

std::vector<int> Executor::table_begins(int launch) const {
  std::vector<int> v;
  if (!rc_ || launch == 1) return v;
  const TableArgs& ta = launch == 0 ? rc_.ta_fwd : rc_.ta_dw;
  for (int i = 0; i < ta.nprob; ++i) v.push_back(ta.begin[i] * c_.R);  // linear block ids
  return v;
}

std::vector<int> Executor::launch_cfgs() const {
  std::vector<int> v;
  if (rc_) return {0, -1, 3};  // table launches (64x32 / 64x64 tiles), the row chain (-1)
  if (tl_.on) {
    for (auto& L : tl_.pre) v.push_back(L.cfg);
    v.push_back(-1);  // the tail chain
    for (auto& L : tl_.post) v.push_back(L.cfg);
    return v;
  }
  for (auto& L : fwd_) v.push_back(L.cfg);
  for (auto& L : bwd_) v.push_back(L.cfg);
  return v;
}

void Executor::train_step(hipStream_t s) {
  run_chunk(s, 1);
  if (!persistent()) advance(1, s);   // the persistent chunk's post node advanced the counters
}

void Executor::train_chunk(int nsteps, hipStream_t s) {
  if (nsteps <= 0) return;
  run_chunk(s, nsteps);
  if (!persistent()) advance(nsteps, s);
}

bool Executor::train_chunk_avg(int nsteps, hipStream_t s, float* out, int write_p, double scale, int mode) {
  if (mode == 2) {   // the averaging in the chunk's post node: any persistent fit-granularity plan
    const bool ok = (pm_.on && !pm_.args.sync && !pm_.args.ps_mode) || (dp_.on && !dp_.args.sync && !dp_.args.ps_mode);
    if (nsteps <= 0 || !ok || c_.nparams <= 0 || c_.P == 0) return false;
    const PostAvg pa{out, write_p, scale};
    post_avg_ = &pa;
    try {
      run_chunk(s, nsteps);
    } catch (...) {
      post_avg_ = nullptr;
      throw;
    }
    post_avg_ = nullptr;
    return true;
  }
  // fit granularity on persist.hip only (per-step sync replicas are one model already; the
  // PS hook's masters belong to the server)
  if (nsteps <= 0 || !pm_.on || pm_.args.sync || pm_.args.ps_mode || c_.nparams <= 0 ||
      (long long)c_.R * c_.sP > 0x7fffffffLL / 4)   // buffer offsets of the averaging's loads
    return false;
  PersistArgs avg{};
  avg.avg_p = write_p;
  avg.avg_n = c_.nparams;
  avg.avg_scale = scale;
  avg.avg_out = out;
  pm_.avg = &avg;
  try {
    run_chunk(s, nsteps);
  } catch (...) {
    pm_.avg = nullptr;
    throw;
  }
  pm_.avg = nullptr;
  return true;
}

void Executor::forward_backward(hipStream_t s) {
  if (rc_) {
    run_rowchain(s, 0, true);
    return;
  }
  run(fwd_, s, 0);
  for (auto L : bwd_) {
    for (int i = 0; i < L.ga.nprob; ++i)
      if (L.ga.p[i].kind == PK_DW_UPDATE) L.ga.p[i].kind = PK_DW_GRAD;
    L.ga.step_off = 0;
    check(ea_gemm_grouped(&L.ga, c_.bf16, L.cfg, s), "gemm_grouped(grad)");
  }
}

FlatArgs Executor::flat_args() const {
  FlatArgs a;
  std::memset(&a, 0, sizeof(a));
  a.R = c_.R;
  a.n = c_.nparams;
  a.P = reinterpret_cast<float*>(c_.P);
  a.sP = c_.sP;
  a.G = reinterpret_cast<const float*>(c_.G);
  a.sG = c_.sG;
  a.S = reinterpret_cast<float*>(c_.S);
  a.sS = c_.sS;
  a.op = c_.op;
  a.nseg = (int)c_.layers.size();
  if (a.nseg > MAX_SEG) throw std::invalid_argument("too many layers for the flat kernels");
  for (int i = 0; i < a.nseg; ++i) {
    const LayerCfg& l = c_.layers[i];
    a.seg[i].p_off = l.p_off;
    a.seg[i].K = l.K;
    a.seg[i].N = l.N;
    a.seg[i].has_bias = l.has_bias;
    a.seg[i].wsh_off = l.wsh_off;
    a.seg[i].ldwsh = l.Np;
    a.seg[i].wtsh_off = l.wtsh_off;
    a.seg[i].ldwtsh = l.Kp;
  }
  a.Wsh = reinterpret_cast<void*>(c_.Wsh);
  a.sWsh = c_.sWsh;
  a.wsh_par = c_.wsh_par;
  a.WTsh = reinterpret_cast<void*>(c_.WTsh);
  a.sWTsh = c_.sWTsh;
  a.wtsh_par = c_.wtsh_par;
  a.ctr = reinterpret_cast<long long*>(c_.ctr);
  a.ntrain = reinterpret_cast<const int*>(c_.ntrain);
  a.B = c_.B;
  return a;
}

void Executor::apply(hipStream_t s) {
  FlatArgs a = flat_args();
  check(ea_apply_update(&a, c_.bf16, s), "apply_update");
  advance(1, s);
}

void Executor::refresh_shadows(bool both, hipStream_t s) {
  FlatArgs a = flat_args();
  a.both_parities = both ? 1 : 0;
  check(ea_refresh_shadows(&a, c_.bf16, s), "refresh_shadows");
}

void Executor::refresh_from(const float* src, float* copy, hipStream_t s) {
  FlatArgs a = flat_args();
  a.both_parities = 1;
  a.src = src;
  a.src_copy = copy;
  check(ea_refresh_shadows(&a, c_.bf16, s), "refresh_from");
}

long long Executor::covered_params() const {
  FlatArgs a = flat_args();
  long long t = 0;
  for (int q = 0; q < a.nseg; ++q) t += (long long)a.seg[q].K * a.seg[q].N + (a.seg[q].has_bias ? a.seg[q].N : 0);
  return t;
}

void Executor::reset_epoch(hipStream_t s) {
  check(hipMemsetAsync(reinterpret_cast<void*>(c_.ctr), 0, 2 * sizeof(long long), s), "reset_epoch");
}

void Executor::eval_chunk(long long chunk, const EvalSource& src, hipStream_t s) {
  auto ls = build_forward(true, chunk, &src);
  run(ls, s, 0);
}

int Executor::capture(int nsteps, int mode, hipStream_t s) {
  hipGraph_t g = nullptr;
  hipGraphExec_t e = nullptr;
  check(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
  try {
    if (mode == 0) {
      // one chunk: steps at offsets 0..nsteps-1 from the counter base, then one advance
      // (the persistent plan's post node includes it)
      run_chunk(s, nsteps);
      if (!persistent()) advance(nsteps, s);
    } else {
      for (int i = 0; i < nsteps; ++i) {
        if (mode == 1) forward_backward(s);
        else apply(s);
      }
    }
  } catch (...) {
    hipGraph_t dummy;
    (void)hipStreamEndCapture(s, &dummy);
    throw;
  }
  check(hipStreamEndCapture(s, &g), "hipStreamEndCapture");
  check(hipGraphInstantiate(&e, g, nullptr, nullptr, 0), "hipGraphInstantiate");
  graphs_.push_back({g, e});
  return (int)graphs_.size() - 1;
}

void Executor::replay(int id, hipStream_t s) {
  if (id < 0 || id >= (int)graphs_.size()) throw std::out_of_range("graph id");
  check(hipGraphLaunch(graphs_[id].second, s), "hipGraphLaunch");
}

}  // namespace ea
