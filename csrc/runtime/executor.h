// Native MLP training executor (MI355X / HIP).
//
// Replaces the reference's per-partition Keras `model.fit` hot loop
// (reference elephas/worker.py:26-49 SparkWorker.train, :76-131
// AsynchronousSparkWorker.train) with a plan of grouped MFMA launches:
//
//   grouped plan:   [FWD_0 + gather X^T] [FWD_1] ... [FWD_{L-1} + loss]   (L launches)
//                   [DW_{L-1} + DX_{L-1}] ... [DW_0]                      (L launches)
//   row-chain plan  (small MLPs, csrc/kernels/rowchain.hip; 3 launches):
//                   [layer-0 split-K slabs + gather X^T] [row chain: layers 1..L-1
//                   forward, loss, dZ_{L-1} .. dZ_0] [DW of every layer]
//   tail-chain plan (deeper stacks whose last two layers fit a 512-wide row chain,
//                   e.g. Otto 93-512-512-512-9): [FWD_0 + gather X^T] .. [FWD_{L-2}]
//                   [chain: layer L-1 forward, loss, dZ_{L-1}, dZ_{L-2}]
//                   [DW_{L-2} + DW_{L-1}] [DX_{L-2}] .. [DW_0] -- the loss launch and
//                   the last layer's backward launch of the grouped plan disappear
//   persistent plan (3-layer MLPs with 64/128-wide hidden layers, fp32;
//                   csrc/kernels/persist.hip): a whole chunk of steps in ONE launch
//                   (+ a 1-block post kernel: flag clear and counter advance)
//   persistent layer pipeline (2..5 Dense layers, hidden widths <= 1024, B <= 128, fp32,
//                   e.g. Otto 93-512-512-512-9; csrc/kernels/deep.hip): the same, with
//                   the replica's workgroups owning column / row tiles of every layer
//
// The step reads its batch index, dropout counter and optimizer iteration from
// device counters, so one captured hipGraph of a step is replayed for every
// step of every epoch (no host round-trip, no per-step launch cost beyond the
// graph's kernel boundaries). R independent replicas ("logical workers" in the
// reference's sense, one per Spark partition) are batched into every launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/args.h"

namespace ea {

struct LayerCfg {
  int K = 0, N = 0, Kp = 0, Np = 0, act = 0, has_bias = 1;
  float rate = 0.f;
  long long p_off = 0;
  uintptr_t Z = 0, D = 0, DT = 0, dZ = 0, dZT = 0;
  long long wsh_off = 0, wtsh_off = 0;
};

struct ExecCfg {
  int R = 1, B = 32, Bp = 32, bf16 = 1;
  unsigned long long seed = 0;
  std::vector<LayerCfg> layers;
  // training data (device)
  uintptr_t X = 0; long long sX = 0, ldx = 0;
  uintptr_t Y = 0; long long sY = 0, ldy = 0;
  uintptr_t perm = 0; long long sPerm = 0;
  uintptr_t ntrain = 0, vstart = 0, vcount = 0;
  uintptr_t XT = 0;
  // parameters
  uintptr_t P = 0; long long sP = 0, nparams = 0;
  uintptr_t G = 0; long long sG = 0;
  uintptr_t S = 0; long long sS = 0;
  uintptr_t Wsh = 0; long long sWsh = 0, wsh_par = 0;
  uintptr_t WTsh = 0; long long sWTsh = 0, wtsh_par = 0;
  OptParams op{};
  int loss = 0, nmet = 0, met[4] = {0, 0, 0, 0};
  uintptr_t acc = 0; int acc_stride = 6;
  uintptr_t ctr = 0;
  int force_cfg = -1;  // -1 auto, 0 LAT, 1 THR, 2 THR-N64, 4 BIG (256x256, bf16)
  int big = 0;         // allow the 256x256 tile where its grid fills the chip (opt-in: measured slower on the Wide shapes)
  int thr_min_n = 256;
  int thr_min_k = 64;  // smallest reduction depth for the 128-row THR tiles (Otto DW, K = batch 128: 135 -> 127 us/step)
  int rowchain = -1;   // row-chain step plan: -1 when eligible, 0 off, 1 required
  int rc_lean = 1;     // skip the update of layer 0's row-major weight image (no reader)
  int rc_split = 0;    // layer-0 split-K slabs of the row-chain plan (0 = auto)
  int tail = -1;       // tail-chain plan when the row chain is not eligible: -1 when eligible, 0 off
  int persist = -1;    // persistent chunk kernel (persist.hip): -1 when eligible, 0 off, 1 required
  long long persist_timeout_ms = 2000;  // spin limit of its in-launch waits
  int persist_cus = 0;  // > 0: CUs the persistent grid may occupy (several executors side by side)
  int persist_v2 = -1;  // persistent V2 roles when eligible (plain SGD, ReLU, independent replicas); 0 off
  int persist_local = -1;  // XCD-local persistent instance where the placement allows (persist_local.hip); 0 off
  int persist_sync = 0;  // persistent plan as per-step synchronous DP of the R replicas (in-launch exchange)
  int deep = -1;        // persistent layer pipeline (deep.hip) where persist.hip is not eligible: -1 when eligible, 0 off,
                        // 2 preferred over persist.hip (tests, A/B)
  int no_reorder = 0;   // A/B: keep a DW + DX launch's problems in declaration order
  int dual = 1;         // a layer's DW and DX on different tiles in one launch (0: two launches)
};

struct EvalSource {
  uintptr_t X = 0; long long sX = 0, ldx = 0;
  uintptr_t Y = 0; long long sY = 0, ldy = 0;
  uintptr_t vstart = 0, vcount = 0;
  uintptr_t acc = 0;
  uintptr_t pred = 0; long long sPred = 0, ldp = 0;
};

class Executor {
 public:
  explicit Executor(const ExecCfg& cfg);
  ~Executor();

  // eager launches on `stream`
  void train_step(hipStream_t s);          // fused-update path (+ counter advance)
  // nsteps fused-update steps (+ one counter advance): ONE launch on the persistent
  // plan whatever nsteps is (no graph needed: memset + kernel + advance)
  void train_chunk(int nsteps, hipStream_t s);
  // the same, on the persistent replica-cluster plan with the replica averaging fused into the
  // launch's end (persist.hip grid_average): scale * sum_r P_r -> out (if not null) and every
  // replica's P (if write_p).  false (nothing launched): the plan cannot -- the caller runs
  // train_chunk and its own averaging
  // mode 1: inside the kernel (persist.hip grid_average, V1 / V2 roles only); mode 2: in the
  // chunk's post node (persist_post_average_kernel: one launch with the flag clear and the
  // counter advance; V1 / V2 roles and the layer pipeline)
  bool train_chunk_avg(int nsteps, hipStream_t s, float* out, int write_p, double scale, int mode = 1);
  void forward_backward(hipStream_t s);    // gradient path: writes G (no update)
  void apply(hipStream_t s);               // gradient path: optimizer apply + advance
  void eval_chunk(long long chunk, const EvalSource& src, hipStream_t s);
  void refresh_shadows(bool both, hipStream_t s);
  // P[r] and both shadow parities of every replica rebuilt from src (a parameter-server
  // pull fused with the refresh); replica 0 also writes src into copy (may be null)
  void refresh_from(const float* src, float* copy, hipStream_t s);
  long long covered_params() const;  // parameters the shadow segments cover
  void reset_epoch(hipStream_t s);

  // hipGraph capture / replay of `nsteps` training steps (mode 0: train_step,
  // mode 1: forward_backward only, mode 2: apply only)
  int capture(int nsteps, int mode, hipStream_t s);
  void replay(int graph_id, hipStream_t s);
  void destroy_graphs();
  void set_seed(unsigned long long seed);   // new dropout seed everywhere (drops captured graphs)

  // launches per step (a captured chunk adds one 1-block counter advance)
  int launches_per_step() const {
    if (rc_.on) return 3;
    if (tl_.on) return (int)tl_.pre.size() + 1 + (int)tl_.post.size();
    return (int)fwd_.size() + (int)bwd_.size();
  }
  bool rowchain() const { return rc_.on; }
  bool tailchain() const { return tl_.on; }
  bool persistent() const { return pm_.on || dp_.on; }
  // persistent plan: {L0 k-chunks, L0 column blocks, k-chunk rows, block columns, chain
  // workgroups, workgroups per replica, grid}
  std::vector<int> persist_geometry() const;
  std::vector<int> persist_variant() const;   // {1 or 2, DW workgroups per replica, sync}
  bool persist_images() const { return pm_.on && pm_.args.imgs != 0; }   // epilogue writes the weight images
  // persistent layer pipeline: {workgroups per replica, grid, row tiles, k-split, LDS bytes}
  std::vector<int> deep_geometry() const;
  // why this executor does not run a persistent plan ("" when it does, or was not asked to)
  std::string plan_reason() const {
    if (persistent() || c_.persist == 0) return "";
    return why_pm_ + (why_dp_.empty() ? "" : "; " + why_dp_);
  }
  // parameter-server hook of the persistent plan (V1 roles only): every step pushes the
  // owned parameters' deltas into the server and pulls the next step's (mode 1 hogwild,
  // 2 asynchronous, 0 off); false when the plan cannot (not persistent, or V2 roles)
  bool set_param_server(const PsArgs& ps, int mode);
  // per-step sync across ranks inside the launch (PersistArgs::xr_*): every rank's
  // rank-exchange buffer (peer-mapped); false: the plan cannot (not a persistent sync plan)
  bool set_rank_exchange(const std::vector<char*>& bases, int world, int rank, unsigned tag0, double timeout_s);
  unsigned rank_exchange_steps() const { return dp_.on ? dp_.xr_steps : pm_.xr_steps; }
  // numeric self-test of the attached exchange: {wrong workgroup-steps, timed-out workgroups}
  std::vector<unsigned> rank_exchange_selftest(int nsteps, int corrupt);
  unsigned persist_error() const;  // sticky error word (a timed-out in-launch wait), synchronous read
  void persist_clear_error();
  int rowchain_split() const { return rc_.on ? rc_.nsplitk : 0; }
  std::vector<int> launch_cfgs() const;
  // diagnostics: bind a [blocks_max][16] int64 buffer for in-kernel stamps (0 = off)
  void set_stamps(uintptr_t buf);
  void train_launch(int idx, hipStream_t s);
  // gradient path one launch at a time (bucketed all-reduce overlapped with the
  // backward): launches [0, nf) are the forward, then one per layer from the last
  // layer down; grad_launch_layer(i) = the layer whose dW / db launch i completes (-1: none)
  int grad_launches() const { return (int)fwd_.size() + (int)bwd_.size(); }
  int grad_launch_layer(int idx) const;
  void grad_launch(int idx, hipStream_t s);
  std::vector<int> launch_blocks() const;
  // row-chain plan: first block of every problem of table launch i (0: A, 2: C)
  std::vector<int> table_begins(int launch) const;

 private:
  struct Launch {
    GroupArgs ga;
    int cfg;
  };
  ExecCfg c_;
  std::vector<Launch> fwd_, bwd_;
  // row-chain plan: table launch A {layer-0 partial slabs, X^T gather}, row chain B,
  // table launch C {DW of every layer} (update, or gradient for the all-reduce path)
  struct RowChain {
    bool on = false;
    int nbw = 2, nsplitk = 1;
    TableArgs ta_fwd{}, ta_dw{}, ta_grad{};
    RcArgs rc{};
    explicit operator bool() const { return on; }
  } rc_;
  Prob* d_probs_ = nullptr;   // device tables of the row-chain launches
  float* d_zp_ = nullptr;     // layer-0 split-K slabs [R][nsplitk][B][N0]
  mutable float* d_zw_ = nullptr;  // (allocated by the const plan builder) wide last layer split-K logit slabs [R][ks][B][N_last]
  bool build_rowchain();
  void run_rowchain(hipStream_t s, int step_off, bool grad) const;
  void make_table(TableArgs& ta, Prob* host, int n, Prob* dev, int cfg) const;
  // tail-chain plan: grouped launches before the chain, the chain, grouped launches
  // after it
  struct Tail {
    bool on = false;
    int nbw = 8;
    std::vector<Launch> pre, post;
    RcArgs rc{};
  } tl_;
  bool build_tail();
  void run_tail(hipStream_t s, int step_off) const;
  struct Persist {
    bool on = false;
    PersistArgs args{};
    size_t flag_bytes = 0;
    mutable unsigned xr_steps = 0;   // steps run with the rank exchange (its flag tags)
    int local = 0;                   // 1: XCD-local instance (ea_persist_local), 2: exchange-local (ea_persist_xlocal)
    mutable PersistArgs* avg = nullptr;   // train_chunk_avg: the averaging fields of the next launch
  } pm_;
  float* d_pws_ = nullptr;         // persistent plan: per-replica exchange workspace
  unsigned* d_pflags_ = nullptr;   // [R][PMF_N][PM_MAXWG] flags (zero at every launch: setup, then the post kernel)
  unsigned* d_perr_ = nullptr;     // sticky error word
  struct PostAvg {
    float* out;
    int write_p;
    double scale;
  };
  mutable const PostAvg* post_avg_ = nullptr;   // train_chunk_avg mode 2: the next chunk's post node averages
  void chunk_post(unsigned* flags, size_t flag_bytes, int nsteps, hipStream_t s) const;
  bool build_persist();
  // persistent layer pipeline (deep.hip)
  struct Deep {
    bool on = false;
    DeepArgs args{};
    size_t flag_bytes = 0;
    mutable unsigned xr_steps = 0;   // steps run with the rank exchange (its flag tags)
    bool local = false;              // the XCD-local instances (deep_l*_local.hip)
  } dp_;
  float* d_dws_ = nullptr;         // its per-replica workspace (activations, gradients, weight images)
  float* d_dxg_ = nullptr;         // its exchange buffer (per-step synchronous replicas)
  unsigned* d_dflags_ = nullptr;   // [R][2][DP_MAXWG] GO / phase counters
  bool build_deep();
  std::string why_pm_, why_dp_;   // why the persistent plans were not eligible (plan_reason)
  void run_chunk(hipStream_t s, int nsteps) const;   // nsteps training steps (no counter advance)
  void run_step(hipStream_t s, int step_off) const;
  std::vector<std::pair<hipGraph_t, hipGraphExec_t>> graphs_;

  Prob base_prob() const;
  void finalize(Launch& L) const;
  int pick_cfg(long long M, long long N, long long K) const;
  int split_last(int cfg, long long N, long long K) const;
  std::vector<Launch> build_forward(bool eval, long long chunk, const EvalSource* src) const;
  void build();
  void run(const std::vector<Launch>& ls, hipStream_t s, int step_off) const;
  void advance(int nsteps, hipStream_t s) const;
  FlatArgs flat_args() const;
};

}  // namespace ea
