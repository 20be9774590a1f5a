// pybind11 bindings for the elephas_amd native runtime (_C).
//
// Tensors cross the boundary as raw device pointers + strides (the Python side
// owns storage through torch's caching allocator) and streams as raw
// hipStream_t handles (torch.cuda.current_stream().cuda_stream), so no torch
// headers or ABI are involved and every launch lands on the caller's stream.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "executor.h"
#include "rwlock.h"
#include "peer.h"
#include "host_loader.h"

namespace py = pybind11;
using namespace ea;

extern "C" hipError_t ea_gemm_grouped(const ea::GroupArgs* ga, int bf16, int cfg, hipStream_t s);
extern "C" int ea_gemm_tile_m(int cfg);
extern "C" int ea_gemm_tile_n(int cfg);
extern "C" void ea_gemm_init();
extern "C" hipError_t ea_replica_average(float* P, long long sP, int R, long long n, float* out, int write_back,
                                         double scale, hipStream_t s);
extern "C" hipError_t ea_axpby(const float* x, float* y, long long n, float alpha, float beta, hipStream_t s);
extern "C" hipError_t ea_sum_slabs(const float* S, int ks, int M, int N, float* C, long long ldc, hipStream_t s);
extern "C" hipError_t ea_ps_sub(float* p, const float* d, long long n, float scale, int atomic, hipStream_t s);
extern "C" hipError_t ea_poison_lds(unsigned pattern, hipStream_t s);
extern "C" hipError_t ea_sub(const float* a, const float* b, float* out, long long n, hipStream_t s);
extern "C" hipError_t ea_shuffle_perm(int* perm, long long sPerm, const int* ntrain, int R, int nmax, uint32_t key,
                                      int shuffle, hipStream_t s);

static void chk(hipError_t e, const char* w) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + w + ": " + hipGetErrorString(e));
}

template <typename T>
static T get(const py::dict& d, const char* k, T def) {
  if (!d.contains(k)) return def;
  py::object o = d[k];
  if (o.is_none()) return def;
  return o.cast<T>();
}

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static OptParams parse_opt(const py::dict& d) {
  OptParams o{};
  o.opt = get<int>(d, "opt", 0);
  o.nesterov = get<int>(d, "nesterov", 0);
  o.lr = get<float>(d, "lr", 0.01f);
  o.decay = get<float>(d, "decay", 0.f);
  o.mom = get<float>(d, "momentum", 0.f);
  o.b1 = get<float>(d, "beta_1", 0.9f);
  o.b2 = get<float>(d, "beta_2", 0.999f);
  o.eps = get<float>(d, "epsilon", 1e-7f);
  o.rho = get<float>(d, "rho", 0.9f);
  o.grad_scale = get<float>(d, "grad_scale", 1.f);
  o.s_plane = get<long long>(d, "s_plane", 0);
  return o;
}

static ExecCfg parse_cfg(const py::dict& d) {
  ExecCfg c;
  c.R = get<int>(d, "R", 1);
  c.B = get<int>(d, "B", 32);
  c.Bp = get<int>(d, "Bp", 32);
  c.bf16 = get<int>(d, "bf16", 1);
  c.seed = get<unsigned long long>(d, "seed", 0);
  c.force_cfg = get<int>(d, "force_cfg", -1);
  c.big = get<int>(d, "big", 0);
  c.rc_lean = get<int>(d, "rc_lean", 1);
  c.thr_min_k = get<int>(d, "thr_min_k", 64);
  c.thr_min_n = get<int>(d, "thr_min_n", 256);
  c.rowchain = get<int>(d, "rowchain", -1);
  c.rc_split = get<int>(d, "rc_split", 0);
  c.tail = get<int>(d, "tail", -1);
  c.no_reorder = get<int>(d, "no_reorder", 0);
  c.dual = get<int>(d, "dual", 1);
  c.persist = get<int>(d, "persist", -1);
  c.persist_timeout_ms = get<long long>(d, "persist_timeout_ms", 2000);
  c.persist_cus = get<int>(d, "persist_cus", 0);
  c.persist_v2 = get<int>(d, "persist_v2", -1);
  c.persist_local = get<int>(d, "persist_local", -1);
  c.persist_sync = get<int>(d, "persist_sync", 0);
  c.deep = get<int>(d, "deep", -1);
  for (auto item : d["layers"].cast<py::list>()) {
    py::dict l = item.cast<py::dict>();
    LayerCfg lc;
    lc.K = get<int>(l, "K", 0);
    lc.N = get<int>(l, "N", 0);
    lc.Kp = get<int>(l, "Kp", 0);
    lc.Np = get<int>(l, "Np", 0);
    lc.act = get<int>(l, "act", 0);
    lc.has_bias = get<int>(l, "has_bias", 1);
    lc.rate = get<float>(l, "rate", 0.f);
    lc.p_off = get<long long>(l, "p_off", 0);
    lc.Z = get<uintptr_t>(l, "Z", 0);
    lc.D = get<uintptr_t>(l, "D", 0);
    lc.DT = get<uintptr_t>(l, "DT", 0);
    lc.dZ = get<uintptr_t>(l, "dZ", 0);
    lc.dZT = get<uintptr_t>(l, "dZT", 0);
    lc.wsh_off = get<long long>(l, "wsh_off", 0);
    lc.wtsh_off = get<long long>(l, "wtsh_off", 0);
    c.layers.push_back(lc);
  }
  c.X = get<uintptr_t>(d, "X", 0);
  c.sX = get<long long>(d, "sX", 0);
  c.ldx = get<long long>(d, "ldx", 0);
  c.Y = get<uintptr_t>(d, "Y", 0);
  c.sY = get<long long>(d, "sY", 0);
  c.ldy = get<long long>(d, "ldy", 0);
  c.perm = get<uintptr_t>(d, "perm", 0);
  c.sPerm = get<long long>(d, "sPerm", 0);
  c.ntrain = get<uintptr_t>(d, "ntrain", 0);
  c.vstart = get<uintptr_t>(d, "vstart", 0);
  c.vcount = get<uintptr_t>(d, "vcount", 0);
  c.XT = get<uintptr_t>(d, "XT", 0);
  c.P = get<uintptr_t>(d, "P", 0);
  c.sP = get<long long>(d, "sP", 0);
  c.nparams = get<long long>(d, "nparams", 0);
  c.G = get<uintptr_t>(d, "G", 0);
  c.sG = get<long long>(d, "sG", 0);
  c.S = get<uintptr_t>(d, "S", 0);
  c.sS = get<long long>(d, "sS", 0);
  c.Wsh = get<uintptr_t>(d, "Wsh", 0);
  c.sWsh = get<long long>(d, "sWsh", 0);
  c.wsh_par = get<long long>(d, "wsh_par", 0);
  c.WTsh = get<uintptr_t>(d, "WTsh", 0);
  c.sWTsh = get<long long>(d, "sWTsh", 0);
  c.wtsh_par = get<long long>(d, "wtsh_par", 0);
  c.op = parse_opt(d["opt"].cast<py::dict>());
  c.loss = get<int>(d, "loss", 0);
  auto mets = get<std::vector<int>>(d, "metrics", {});
  if (mets.size() > 4) throw std::invalid_argument("at most 4 fused metrics");
  c.nmet = (int)mets.size();
  for (size_t i = 0; i < mets.size(); ++i) c.met[i] = mets[i];
  c.acc = get<uintptr_t>(d, "acc", 0);
  c.acc_stride = get<int>(d, "acc_stride", 6);
  c.ctr = get<uintptr_t>(d, "ctr", 0);
  return c;
}

static EvalSource parse_src(const py::dict& d) {
  EvalSource e;
  e.X = get<uintptr_t>(d, "X", 0);
  e.sX = get<long long>(d, "sX", 0);
  e.ldx = get<long long>(d, "ldx", 0);
  e.Y = get<uintptr_t>(d, "Y", 0);
  e.sY = get<long long>(d, "sY", 0);
  e.ldy = get<long long>(d, "ldy", 0);
  e.vstart = get<uintptr_t>(d, "vstart", 0);
  e.vcount = get<uintptr_t>(d, "vcount", 0);
  e.acc = get<uintptr_t>(d, "acc", 0);
  e.pred = get<uintptr_t>(d, "pred", 0);
  e.sPred = get<long long>(d, "sPred", 0);
  e.ldp = get<long long>(d, "ldp", 0);
  return e;
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "elephas_amd native runtime: CDNA4 (gfx950) HIP kernels + executor";
#ifndef EA_SRC_DIGEST
#define EA_SRC_DIGEST "unknown"
#endif
  // sha256 prefix of the csrc/ sources this binary was built from (elephas_amd/_build.py)
  m.attr("source_digest") = EA_SRC_DIGEST;

  py::class_<Executor>(m, "Executor")
      .def(py::init([](py::dict cfg) { return new Executor(parse_cfg(cfg)); }))
      .def("train_step", [](Executor& e, uintptr_t s) { e.train_step(S(s)); })
      .def("train_chunk", [](Executor& e, int n, uintptr_t s) { e.train_chunk(n, S(s)); })
      .def("train_chunk_avg", [](Executor& e, int n, uintptr_t s, uintptr_t out, int write_p, double scale, int mode) {
        return e.train_chunk_avg(n, S(s), reinterpret_cast<float*>(out), write_p, scale, mode);
      })
      .def("forward_backward", [](Executor& e, uintptr_t s) { e.forward_backward(S(s)); })
      .def("apply", [](Executor& e, uintptr_t s) { e.apply(S(s)); })
      .def("eval_chunk", [](Executor& e, long long chunk, py::dict src, uintptr_t s) {
        e.eval_chunk(chunk, parse_src(src), S(s));
      })
      .def("refresh_shadows", [](Executor& e, bool both, uintptr_t s) { e.refresh_shadows(both, S(s)); })
      .def("reset_epoch", [](Executor& e, uintptr_t s) { e.reset_epoch(S(s)); })
      .def("refresh_from", [](Executor& e, uintptr_t src, uintptr_t copy, uintptr_t s) {
        e.refresh_from(reinterpret_cast<const float*>(src), reinterpret_cast<float*>(copy), S(s));
      })
      .def("capture", [](Executor& e, int n, int mode, uintptr_t s) { return e.capture(n, mode, S(s)); })
      .def("replay", [](Executor& e, int id, uintptr_t s) {
        py::gil_scoped_release rel;
        e.replay(id, S(s));
      })
      .def("replay_n", [](Executor& e, int id, int times, uintptr_t s) {
        py::gil_scoped_release rel;
        for (int i = 0; i < times; ++i) e.replay(id, S(s));
      })
      .def("destroy_graphs", &Executor::destroy_graphs)
      .def("launches_per_step", &Executor::launches_per_step)
      .def("launch_cfgs", &Executor::launch_cfgs)
      .def("launch_blocks", &Executor::launch_blocks)
      .def("table_begins", &Executor::table_begins)
      .def("rowchain", &Executor::rowchain)
      .def("rowchain_split", &Executor::rowchain_split)
      .def("tailchain", &Executor::tailchain)
      .def("persistent", &Executor::persistent)
      .def("persist_geometry", &Executor::persist_geometry)
      .def("persist_variant", &Executor::persist_variant)
      .def("deep_geometry", &Executor::deep_geometry)
      .def("set_seed", &Executor::set_seed)
      .def("plan_reason", &Executor::plan_reason)
      .def("rank_exchange_selftest", &Executor::rank_exchange_selftest)
      .def("persist_images", &Executor::persist_images)
      .def("set_rank_exchange", [](Executor& e, std::vector<uintptr_t> bases, int world, int rank, unsigned tag0,
                                   double timeout_s) {
        std::vector<char*> b;
        for (auto p : bases) b.push_back(reinterpret_cast<char*>(p));
        return e.set_rank_exchange(b, world, rank, tag0, timeout_s);
      })
      .def("rank_exchange_steps", &Executor::rank_exchange_steps)
      .def("set_param_server", [](Executor& e, ShardedParameterServer* ps, int mode) {
        return e.set_param_server(ps ? ps->kernel_args() : PsArgs{}, ps ? mode : 0);
      }, py::arg("ps"), py::arg("mode"))
      .def("persist_error", &Executor::persist_error)
      .def("persist_clear_error", &Executor::persist_clear_error)
      .def("set_stamps", &Executor::set_stamps)
      .def("train_launch", [](Executor& e, int idx, uintptr_t s) { e.train_launch(idx, S(s)); })
      .def("grad_launches", &Executor::grad_launches)
      .def("grad_launch_layer", &Executor::grad_launch_layer)
      .def("grad_launch", [](Executor& e, int idx, uintptr_t s) { e.grad_launch(idx, S(s)); });

  // single PLAIN GEMM (C fp32 = A . BT^T) for kernel tests / generic matmul
  // splitk > 1 (fp32 C only): the reduction split over splitk workgroup slabs (PK_PARTIAL, the
  // Wide model's last-layer form), then one slab-sum launch -- for grids too small to fill the
  // 256 CUs (1024 x 1000 x 4096: 64 tiles of 128 x 128)
  m.def("gemm_nt", [](uintptr_t A, uintptr_t BT, uintptr_t C, int M, int N, int K, long long lda, long long ldb,
                      long long ldc, int bf16, int cfg, uintptr_t s, uintptr_t stamps, int out_bf16, int splitk) {
    // the kernel issues unconditional 16-byte fragment loads along K: rows must be
    // 16-byte aligned and K padded to whole chunks, or it reads out of bounds
    const int epl = bf16 ? 8 : 4;
    if (M <= 0 || N <= 0 || K <= 0 || (K % epl) || (lda % epl) || (ldb % epl) || lda < K || ldb < K || ldc < N ||
        (A % 16) || (BT % 16) || (C % 4) || cfg < 0 || cfg > 7 || cfg == 3)
      throw std::invalid_argument("gemm_nt: K, lda, ldb must be multiples of 16 bytes, pointers 16-byte aligned");
    ea_gemm_init();
    if (cfg >= 4 && !bf16) cfg = 1;  // the 256x256 tiles are bf16-only; fp32 runs the THR tile
    GroupArgs ga;
    std::memset(&ga, 0, sizeof(ga));
    Prob& p = ga.p[0];
    p.kind = PK_PLAIN;
    p.M = M; p.N = N; p.K = K; p.R = 1;
    p.A = reinterpret_cast<const void*>(A); p.lda = lda;
    p.BT = reinterpret_cast<const void*>(BT); p.ldb = ldb;
    p.D = reinterpret_cast<void*>(C); p.ldd = ldc;
    p.d_bf16 = out_bf16 ? 1 : 0;   // C holds bf16 (16-byte aligned rows for the vector stores)
    p.ones_row = -1;
    p.B = M;
    p.tiles_m = (M + ea_gemm_tile_m(cfg) - 1) / ea_gemm_tile_m(cfg);
    p.tiles_n = (N + ea_gemm_tile_n(cfg) - 1) / ea_gemm_tile_n(cfg);
    ga.nprob = 1;
    ga.R = 1;
    ga.total_blocks = p.tiles_m * p.tiles_n;
    ga.stamps = reinterpret_cast<long long*>(stamps);  // diagnostics (null = off)
    static float* slabs = nullptr;
    static size_t slab_cap = 0;
    if (splitk > 1) {
      if (out_bf16 || splitk > 16) throw std::invalid_argument("gemm_nt: splitk needs fp32 C and <= 16 slabs");
      const size_t need = (size_t)splitk * M * N;
      if (need > slab_cap) {
        if (slabs) chk(hipFree(slabs), "hipFree");
        chk(hipMalloc(&slabs, need * sizeof(float)), "hipMalloc(split-K slabs)");
        slab_cap = need;
      }
      p.kind = PK_PARTIAL;
      p.tiles_k = splitk;
      p.kchunk = ((K + splitk - 1) / splitk + 63) / 64 * 64;
      p.D = slabs;
      p.ldd = N;
      p.sPart = (long long)M * N;
      p.sD = (long long)splitk * M * N;
      ga.total_blocks *= splitk;
    }
    static long long* dctr = nullptr;
    if (!dctr) {
      chk(hipMalloc(&dctr, 64 * sizeof(long long)), "hipMalloc");
      chk(hipMemset(dctr, 0, 64 * sizeof(long long)), "hipMemset");
    }
    ga.ctr = dctr;
    p.ntrain = reinterpret_cast<const int*>(dctr);  // zero batch counts: the kernel reads ntrain[0]
    chk(ea_gemm_grouped(&ga, bf16, cfg, S(s)), "gemm_nt");
    if (splitk > 1) chk(ea_sum_slabs(slabs, splitk, M, N, reinterpret_cast<float*>(C), ldc, S(s)), "gemm_nt slab sum");
  }, py::arg("A"), py::arg("BT"), py::arg("C"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("lda"),
     py::arg("ldb"), py::arg("ldc"), py::arg("bf16"), py::arg("cfg"), py::arg("stream"), py::arg("stamps") = 0,
     py::arg("out_bf16") = 0, py::arg("splitk") = 1);
  m.def("tile_shape", [](int cfg) { return py::make_tuple(ea_gemm_tile_m(cfg), ea_gemm_tile_n(cfg)); });

  m.def("replica_average", [](uintptr_t P, long long sP, int R, long long n, uintptr_t out, int write_back,
                              uintptr_t s, double scale) {
    // scale <= 0: the mean (1 / R); 1.0: the plain sum (the multi-rank averaging path)
    chk(ea_replica_average(reinterpret_cast<float*>(P), sP, R, n, reinterpret_cast<float*>(out), write_back,
                           scale > 0.0 ? scale : 1.0 / R, S(s)),
        "replica_average");
  }, py::arg("P"), py::arg("sP"), py::arg("R"), py::arg("n"), py::arg("out"), py::arg("write_back"), py::arg("stream"),
     py::arg("scale") = 0.0);
  m.def("shuffle_perm", [](uintptr_t perm, long long sPerm, uintptr_t ntrain, int R, int nmax, uint32_t key,
                           int shuffle, uintptr_t s) {
    // per-replica keyed Feistel permutation of rows [0, ntrain[r]) (csrc/kernels/shuffle.hip)
    chk(ea_shuffle_perm(reinterpret_cast<int*>(perm), sPerm, reinterpret_cast<const int*>(ntrain), R, nmax, key,
                        shuffle, S(s)),
        "shuffle_perm");
  }, py::arg("perm"), py::arg("sPerm"), py::arg("ntrain"), py::arg("R"), py::arg("nmax"), py::arg("key"),
     py::arg("shuffle"), py::arg("stream"));
  m.def("axpby", [](uintptr_t x, uintptr_t y, long long n, float a, float b, uintptr_t s) {
    chk(ea_axpby(reinterpret_cast<const float*>(x), reinterpret_cast<float*>(y), n, a, b, S(s)), "axpby");
  });
  m.def("ps_sub", [](uintptr_t p, uintptr_t d, long long n, float scale, int atomic, uintptr_t s) {
    chk(ea_ps_sub(reinterpret_cast<float*>(p), reinterpret_cast<const float*>(d), n, scale, atomic, S(s)), "ps_sub");
  });
  m.def("poison_lds", [](unsigned pattern, uintptr_t s) { chk(ea_poison_lds(pattern, S(s)), "poison_lds"); });
  m.def("sub", [](uintptr_t a, uintptr_t b, uintptr_t out, long long n, uintptr_t s) {
    chk(ea_sub(reinterpret_cast<const float*>(a), reinterpret_cast<const float*>(b), reinterpret_cast<float*>(out), n,
               S(s)),
        "sub");
  });

  // ---- peer-memory collectives and the sharded device PS (peer.h)
  // a bare peer-mapped buffer (the persistent kernel's rank exchange, PersistArgs::xr_*)
  py::class_<PeerBuffer>(m, "PeerBuffer")
      .def(py::init<int, int, long long, int>(), py::arg("rank"), py::arg("world"), py::arg("data_bytes"),
           py::arg("device"))
      .def("handle", [](PeerBuffer& p) { return py::bytes(p.handle()); })
      .def("open", [](PeerBuffer& p, std::vector<py::bytes> hs) {
        std::vector<std::string> v;
        for (auto& h : hs) v.emplace_back(std::string(h));
        p.open(v);
      })
      .def("bases", [](PeerBuffer& p) {
        std::vector<uintptr_t> v;
        for (int r = 0; r < p.world(); ++r) v.push_back(reinterpret_cast<uintptr_t>(p.base(r)));
        return v;
      })
      .def("error", &PeerBuffer::error)
      .def("release", &PeerBuffer::release);

  py::class_<PeerAllReduce>(m, "PeerAllReduce")
      .def(py::init<int, int, long long, int, double>(), py::arg("rank"), py::arg("world"), py::arg("cap_elems"),
           py::arg("device"), py::arg("timeout_s") = 20.0)
      .def("handle", [](PeerAllReduce& p) { return py::bytes(p.handle()); })
      .def("open", [](PeerAllReduce& p, std::vector<py::bytes> hs) {
        std::vector<std::string> v;
        for (auto& h : hs) v.emplace_back(std::string(h));
        p.open(v);
      })
      .def("all_reduce", [](PeerAllReduce& p, uintptr_t in, uintptr_t out, long long n, uintptr_t s, int algo) {
        py::gil_scoped_release rel;
        p.all_reduce(reinterpret_cast<const float*>(in), reinterpret_cast<float*>(out), n, S(s), algo);
      }, py::arg("inp"), py::arg("out"), py::arg("n"), py::arg("stream"), py::arg("algo") = -1)
      .def("all_reduce_graph", [](PeerAllReduce& p, uintptr_t in, uintptr_t out, long long n, uintptr_t s, int algo) {
        p.all_reduce_graph(reinterpret_cast<const float*>(in), reinterpret_cast<float*>(out), n, S(s), algo);
      }, py::arg("inp"), py::arg("out"), py::arg("n"), py::arg("stream"), py::arg("algo") = -1)
      .def("error", &PeerAllReduce::error)
      .def("clear_error", &PeerAllReduce::clear_error)
      .def("release", &PeerAllReduce::release)
      .def_property_readonly("capacity", &PeerAllReduce::capacity)
      .def_property_readonly("calls", &PeerAllReduce::calls)
      .def_property("twoshot_min_bytes", &PeerAllReduce::twoshot_min_bytes, &PeerAllReduce::set_twoshot_min_bytes);
  py::class_<ShardedParameterServer>(m, "ShardedParameterServer")
      .def(py::init<int, int, long long, int, int, long long, double>(), py::arg("rank"), py::arg("world"),
           py::arg("n"), py::arg("consistent"), py::arg("device"), py::arg("chunk") = 4096, py::arg("timeout_s") = 30.0)
      .def("handle", [](ShardedParameterServer& p) { return py::bytes(p.handle()); })
      .def("open", [](ShardedParameterServer& p, std::vector<py::bytes> hs) {
        std::vector<std::string> v;
        for (auto& h : hs) v.emplace_back(std::string(h));
        p.open(v);
      })
      .def("set", [](ShardedParameterServer& p, uintptr_t src, uintptr_t s) {
        p.set(reinterpret_cast<const float*>(src), S(s));
      })
      .def("pull", [](ShardedParameterServer& p, uintptr_t dst, uintptr_t s) {
        p.pull(reinterpret_cast<float*>(dst), S(s));
      })
      .def("pull_replicas", [](ShardedParameterServer& p, uintptr_t dst, uintptr_t P, long long sP, int R, uintptr_t s) {
        p.pull_replicas(reinterpret_cast<float*>(dst), reinterpret_cast<float*>(P), sP, R, S(s));
      })
      .def("push_replicas", [](ShardedParameterServer& p, uintptr_t P, long long sP, int R, uintptr_t before,
                               uintptr_t s) {
        p.push_replicas(reinterpret_cast<const float*>(P), sP, R, reinterpret_cast<const float*>(before), S(s));
      })
      .def("push_delta", [](ShardedParameterServer& p, uintptr_t d, uintptr_t s) {
        p.push_delta(reinterpret_cast<const float*>(d), S(s));
      })
      .def("error", &ShardedParameterServer::error)
      .def("clear_error", &ShardedParameterServer::clear_error)
      .def("release", &ShardedParameterServer::release)
      .def("shard_begin", &ShardedParameterServer::shard_begin)
      .def_property_readonly("n", &ShardedParameterServer::size)
      .def_property_readonly("consistent", &ShardedParameterServer::consistent)
      .def_property_readonly("nchunks", &ShardedParameterServer::nchunks);
  m.def("shm_rwlock_create", &shm_rwlock_create);
  m.def("shm_rwlock_destroy", &shm_rwlock_destroy);

  // ---- host loader (pinned, double-buffered H2D)
  py::class_<HostLoader>(m, "HostLoader")
      .def(py::init<long long, int, int>(), py::arg("chunk_bytes"), py::arg("nbuf") = 3, py::arg("threads") = 0)
      .def("upload", [](HostLoader& L, uintptr_t host, uintptr_t dev, long long nbytes, uintptr_t s) {
        py::gil_scoped_release rel;
        L.upload(reinterpret_cast<const void*>(host), reinterpret_cast<void*>(dev), nbytes, S(s));
      })
      .def("upload_rows", [](HostLoader& L, uintptr_t host, long long host_ld, uintptr_t dev, long long dev_ld,
                             long long nrows, long long row_bytes, uintptr_t s) {
        py::gil_scoped_release rel;
        L.upload_rows(reinterpret_cast<const char*>(host), host_ld, reinterpret_cast<char*>(dev), dev_ld, nrows,
                      row_bytes, S(s));
      })
      .def("upload_rows_bf16", [](HostLoader& L, uintptr_t host, long long host_ld, uintptr_t dev, long long dev_ld,
                                  long long nrows, long long ncols, uintptr_t s) {
        py::gil_scoped_release rel;
        L.upload_rows_bf16(reinterpret_cast<const float*>(host), host_ld, reinterpret_cast<char*>(dev), dev_ld,
                           nrows, ncols, S(s));
      })
      .def_property_readonly("chunk_bytes", &HostLoader::chunk_bytes)
      .def_property_readonly("bytes_uploaded", &HostLoader::bytes_uploaded)
      .def_property_readonly("threads", &HostLoader::threads)
      .def_property_readonly("last_pack_threads", &HostLoader::last_pack_threads);

  m.def("infer_pipeline", [](Executor& exe, HostLoader& L, py::dict a, py::dict src, uintptr_t s_up, uintptr_t s_comp,
                             uintptr_t s_down) {
    // inference over host rows: staged uploads / eval chunks / prediction downloads on
    // three streams (csrc/runtime/host_loader.h)
    InferPipeArgs p;
    p.x = reinterpret_cast<const float*>(get<uintptr_t>(a, "x", 0));
    p.x_ld = get<long long>(a, "x_ld", 0);
    p.n = get<long long>(a, "n", 0);
    p.k = get<long long>(a, "k", 0);
    p.dX = reinterpret_cast<char*>(get<uintptr_t>(a, "dX", 0));
    p.dX_ld = get<long long>(a, "dX_ld", 0);
    p.x_bf16 = get<int>(a, "x_bf16", 0);
    p.y = reinterpret_cast<const float*>(get<uintptr_t>(a, "y", 0));
    p.y_ld = get<long long>(a, "y_ld", 0);
    p.ky = get<long long>(a, "ky", 0);
    p.dY = reinterpret_cast<float*>(get<uintptr_t>(a, "dY", 0));
    p.dY_ld = get<long long>(a, "dY_ld", 0);
    p.dPred = reinterpret_cast<float*>(get<uintptr_t>(a, "dPred", 0));
    p.ldp = get<long long>(a, "ldp", 0);
    p.hPred = reinterpret_cast<float*>(get<uintptr_t>(a, "hPred", 0));
    p.out = reinterpret_cast<float*>(get<uintptr_t>(a, "out", 0));
    p.dStage = reinterpret_cast<float*>(get<uintptr_t>(a, "dStage", 0));
    p.stage_rows = get<long long>(a, "stage_rows", 0);
    p.B = get<int>(a, "B", 0);
    const EvalSource es = parse_src(src);
    py::gil_scoped_release rel;
    infer_pipeline(exe, L, p, es, S(s_up), S(s_comp), S(s_down));
  });
}
