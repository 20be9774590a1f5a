// Launch-argument structs shared by the device kernels and the native executor
// (csrc/runtime/executor.cpp). Plain-old-data only: passed by value as kernel args.
#pragma once
#include <stdint.h>

#include "peer_args.h"

namespace ea {

// ---------------------------------------------------------------- enums ----
// Keep in sync with elephas_amd/ops/native.py
enum Act : int {
  ACT_LINEAR = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3, ACT_SOFTMAX = 4,
  ACT_ELU = 5, ACT_SELU = 6, ACT_SOFTPLUS = 7, ACT_SOFTSIGN = 8, ACT_EXPONENTIAL = 9,
  ACT_HARD_SIGMOID = 10, ACT_SWISH = 11, ACT_GELU = 12, ACT_RELU6 = 13
};

enum Loss : int {
  LOSS_CCE = 0, LOSS_SPARSE_CCE = 1, LOSS_BCE = 2, LOSS_MSE = 3, LOSS_MAE = 4,
  LOSS_MAPE = 5, LOSS_MSLE = 6, LOSS_LOGCOSH = 7, LOSS_HINGE = 8, LOSS_SQ_HINGE = 9,
  LOSS_KLD = 10, LOSS_POISSON = 11, LOSS_COSINE = 12, LOSS_CAT_HINGE = 13
};

// Metrics: values < 100 reuse the Loss enum (a loss evaluated as a metric);
// accuracies use the 100+ range.
enum Metric : int {
  MET_ACC_CAT = 100, MET_ACC_SPARSE = 101, MET_ACC_BIN = 102
};

enum Opt : int { OPT_SGD = 0, OPT_RMSPROP = 1, OPT_ADAM = 2, OPT_ADAGRAD = 3, OPT_ADAMAX = 4 };

struct OptParams {
  int opt; int nesterov; float lr, decay, mom, b1, b2, eps, rho, grad_scale;
  long long s_plane;  // stride between optimizer state planes (elements)
};

enum ProbKind : int {
  PK_PLAIN = 0,      // C (fp32) = A.BT
  PK_FWD = 1,        // Z = A.BT + b ; D = dropout(act(Z)) ; D^T
  PK_FWD_LOSS = 2,   // final layer: logits -> loss/metrics -> dZ, dZ^T (or predictions)
  PK_DX = 3,         // dZ_{l-1} = (dZ_l.W_l^T) * act'(Z_{l-1}) * mask_{l-1}
  PK_DW_UPDATE = 4,  // dW -> fused optimizer update of master params + bf16/f32 shadows
  PK_DW_GRAD = 5,    // dW -> flat gradient buffer (all-reduce path)
  PK_GATHER_T = 6,   // X^T batch (gathered through perm) for DW of layer 1
  PK_LOSS_ROWS = 7,  // wide final layer: one wave per row over fp32 logits Z
  PK_PARTIAL = 8     // split-K slab: fp32 C over K chunk kc -> D + r*sD + kc*sPart (row-chain layer 0,
                     // wide last layer); a new kind must be added to KM_ALL (gemm_impl.h)
};

struct Prob {
  int kind;
  int M, N, K;             // K: padded reduction length (multiple of 8)
  int R;                   // replicas
  int tiles_m, tiles_n;
  int tiles_k;             // split-K chunks over workgroups (PK_PARTIAL; 1 otherwise)
  int kchunk;              // reduction elements per chunk (multiple of 8)
  long long sPart;         // element stride between the chunks' output slabs
  int block_begin;
  // operands
  const void* A; long long lda, sA;
  const void* BT; long long ldb, sB;
  int a_gather;            // 1: A rows come from the batch window (train: perm, eval: contiguous)
  int ones_row;            // >= 0: index of a virtual all-ones A row (bias gradient)
  int bt_shadow;           // 1: BT is a parity-double-buffered shadow (offset by par * bt_par)
  long long bt_par;
  // batch window
  const int* perm; long long sPerm;
  const int* ntrain;       // per replica number of training rows (0 => replica inactive)
  const int* vstart;       // eval: per replica first row
  const int* vcount;       // eval: per replica number of rows
  int B;                   // rows per step
  int eval_mode;
  long long chunk;         // eval: chunk index (rows chunk*B ...)
  // layer epilogue
  int act; float rate; int layer; int row_valid_mask;
  const float* bias; long long sBias;
  float* Z; long long ldz, sZ;
  void* D; long long ldd, sD;
  int d_bf16;              // PK_PLAIN: D holds bf16 (else fp32)
  void* DT; long long lddt, sDT;
  // loss
  int loss; int nmet; int met[4];
  const float* Y; long long ldy, sY;
  double* acc; int acc_stride;
  float* pred; long long ldp, sPred;
  // parameters / optimizer
  float* P; long long sP; long long p_off;
  float* G; long long sG;
  float* S; long long sS;
  void* Wsh; long long sWsh, ldwsh, wsh_par;
  void* WTsh; long long sWTsh, ldwtsh, wtsh_par;
  OptParams op;
};

struct GroupArgs {
  Prob p[2];
  int nprob;
  // grid (R, total_blocks): blockIdx.x = replica, blockIdx.y = tile of the launch.
  // Blocks are dealt to the 8 XCDs round-robin in x-fastest order, so with R = 8 a
  // replica's tiles share one XCD's L2 (and the replica index is a scalar register:
  // no integer division on the vector ALU)
  int R;
  int total_blocks;   // tiles per replica; problem i owns tiles [p[i].block_begin, ...)
  long long* ctr;           // [0]=step in epoch, [1]=arrive counter, [2..2+R)=iter per replica
  unsigned long long seed;
  // Step counters: ctr[0] = base step-in-epoch, ctr[2 + r] = base optimizer
  // iteration of replica r. Kernels only READ them: a launch at position
  // `step_off` of a captured chunk uses step = ctr[0] + step_off and
  // iter_r = ctr[2+r] + clamp(nb_r - ctr[0], 0, step_off) (nb_r = batches of
  // replica r per epoch); one 1-block advance kernel per chunk moves the base.
  // (No same-address atomics in the step: those serialise at ~60 ns each.)
  int step_off;
  long long* stamps;        // diagnostics: [block][16] s_memrealtime stamps (null = off)
};

// A grouped launch whose problems live in a device table (csrc/runtime/executor.cpp
// row-chain plan): up to TABLE_MAX problems of one kind set, problem i owns blocks
// [begin[i], begin[i+1]). Problem fields are read through the pointer with scalar
// loads (the index is wave-uniform); GroupArgs keeps two problems in kernarg.
constexpr int TABLE_MAX = 4;
struct TableArgs {
  const Prob* probs;
  int nprob;
  int begin[TABLE_MAX];   // first tile (per replica) of every problem
  int R;                  // grid (R, total_blocks) as GroupArgs
  int total_blocks;
  long long* ctr;
  unsigned long long seed;
  int step_off;
  long long* stamps;
};

// --------------------------------------------------------- row-chain MLP step
// Layers 1..L-1 of a small MLP (every width <= RC_MAXW) for RC_ROWS batch rows
// per workgroup: forward, loss, and input gradients (see rowchain.hip).
constexpr int RC_MAXL = 4;
constexpr int RC_ROWS = 16;
constexpr int RC_MAXW = 256;
constexpr int RC_TAILW = 512;    // the tail chain (L = 2: the last two layers of a deeper stack)
constexpr int RC_MAXSPLIT = 8;   // layer-0 split-K slabs
constexpr int LOSS_RPB = 4;        // rows per workgroup of the wide-output loss rows kernel (one per wave)
constexpr int LOSS_MAX_SPLIT = 4;  // split-K slabs of a wide last layer summed by the loss rows kernel
struct RcLayer {
  int K, N, Kp, Np, act, has_bias;
  float rate;
  long long p_off, wsh_off, wtsh_off;
  void* DT;    // D_l^T [N][Bp] (compute dtype), the next layer's DW operand (l < L-1)
  void* dZT;   // dZ_l^T [N][Bp], this layer's DW operand
};
struct RcArgs {
  int L, R, B, Bp;
  int nsplitk;                  // layer-0 split-K partial slabs
  const float* Zp; long long sZp, sZpk;   // [R][nsplitk][B][N0] fp32
  RcLayer ly[RC_MAXL];          // indexed with compile-time layer numbers only
  const float* Y; long long sY, ldy;
  const int* perm; long long sPerm;
  const int* ntrain;
  const float* P; long long sP;            // fp32 master (biases)
  const void* Wsh; long long sWsh, wsh_par;
  const void* WTsh; long long sWTsh, wtsh_par;
  int loss, nmet, met[4];
  double* acc; int acc_stride;
  long long* ctr; int step_off;
  unsigned long long seed;
  long long* stamps;
  // tail chain: the chain's layer 0 is model layer l0 (dropout streams are keyed by
  // model layer) whose pre-activations Zsrc [R][B][ldzs] (fp32, bias included) a grouped
  // FWD launch wrote -- read instead of split-K slabs (null: slabs); dZ_0 also goes out
  // row-major (the A operand of the grouped DX launch below the chain; null = not written)
  int l0;
  const float* Zsrc; long long ldzs;
  void* dZ0; long long ldz0;
};

// ------------------------------------------------- persistent replica-cluster step
// A chunk of training steps of a 3-layer Dense stack (hidden widths 64 or 128, a last
// layer of <= 16 units) in ONE launch (csrc/kernels/persist.hip): per replica, nk0 x nc0
// layer-0 workgroups keep their W0 tile resident in LDS and nch = ceil(B/16) chain
// workgroups run layers 1-2 for 16 batch rows each; they hand activations, gradients
// and updated weights to each other through a per-replica workspace with flags.
constexpr int PM_ROWS = 64;    // batch rows per replica (B <= 64)
constexpr int PM_MAXH = 128;   // hidden widths: 64 or 128
constexpr int PM_MAXC = 16;    // last layer units
constexpr int PM_MAXWG = 64;   // workgroups of one kind per replica (one polling wave watches them)
constexpr int PM_NTU = 2;      // layer-1 column tiles (and layer-2 row tiles) a chain / DW workgroup owns
// hand-off flag kinds: PART (layer-0 partials of a step), BWD (a chain's dZ_0 rows), W
// (updated W1 / W2 columns), A0 / D2 (V2: a chain's layer-0 activations / dZ_2 and
// layer-1 activations for the weight-gradient workgroups), GO (residency: every
// workgroup raises it on entry; the chain workgroups see the whole grid before they
// touch any state)
// X (sync: a workgroup's weight-gradient tile is in the exchange slab, see PersistArgs::sync),
// GR (V2 with ng > 0: a weight-gradient workgroup's Gram slab of a step is out)
// XT (sync across ranks: replica 0's workgroup q has the job-wide sum of its tile in its
// total slab; the other replicas read it there instead of every rank's slab)
enum PmFlag : int { PMF_PART = 0, PMF_BWD = 1, PMF_W = 2, PMF_A0 = 3, PMF_D2 = 4, PMF_GO = 5, PMF_X = 6, PMF_GR = 7,
                    PMF_XT = 8, PMF_XS = 9, PMF_AVG = 10, PMF_N = 11 };
// sticky error codes: the wait that timed out (PERR_GRID: the grid was not resident --
// nothing was modified, the chunk can be re-run on another plan)
enum PmErr : unsigned { PERR_L0_BWD = 1, PERR_CHAIN_PART = 2, PERR_CHAIN_BWD = 3, PERR_CHAIN_PREV = 4,
                        PERR_DW_A0 = 5, PERR_DW_D2 = 6, PERR_XCHG = 7, PERR_PS = 8, PERR_GRID = 9,
                        PERR_CHAIN_GR = 10, PERR_XRANK = 11, PERR_PLACE = 12, PERR_AVG = 13 };
constexpr int PM_XSLOT = 7 * 1024;   // floats of one workgroup's exchange slab (sync)
struct PersistArgs {
  int R, B, nsteps;
  int K0, H0, H1, C;            // layer widths (H0, H1 in {64, 128}; C <= 16)
  int nk0, nc0, kc0, cw;        // layer-0 tiles: nk0 k-chunks of kc0 rows x nc0 column blocks of cw
  int nch, wgs;                 // chain workgroups per replica; workgroups per replica (nk0*nc0 + nch [+ nd])
  // V2 (plain SGD, ReLU, fit granularity): nd weight-gradient workgroups per replica own
  // the W1 columns / W2 rows; the chain rebuilds Z_0 from Pold + Gram corrections
  int v2, nd;
  // V2 Gram slabs X_s . X_{s-1}^T: ng > 0 -- computed by the weight-gradient workgroups
  // d < ng over k-chunks of gk columns (their idle window between W and A0), one slab each;
  // ng = 0 -- by the layer-0 tiles, one slab per k-chunk of kc0 (nk0 slabs)
  int ng, gk;
  long long o_g;                    // Gram partials [3][max(nk0, ng)][64][64] (V2)
  long long part_par, g_par, dz0_par;   // parity strides of the double-buffered partials / Gram / dZ_0 (V2; 0 in V1)
  // sync (V1 roles, per-step synchronous DP of the R replicas = one model): after its
  // weight-gradient MFMAs every owning workgroup puts its tile into its exchange slab
  // (parity of the step), raises X, waits for the same workgroup of every replica and
  // sums the R slabs in replica order -- the same bits everywhere, so the replicas'
  // updates (grad_scale = 1 / R) keep their weights identical
  int sync;
  int xchg_rs;                      // sync: reduce-scatter + all-gather of the slabs (else all-gather + sum)
  long long o_xg;                   // exchange slabs [2][wgs][PM_XSLOT] in every replica's workspace
  // sync across ranks (xr_world > 1; one node, every rank the same step sequence): after
  // the replica sum, replica 0's owning workgroup q puts the rank's sum into slab
  // [tag & 1][q] of its rank-exchange buffer (peer-mapped, uncached; peer_args.h offsets)
  // and raises flag q (system scope, tag = xr_tag0 + step + 1, monotonic over the trainer's
  // life); every replica then sums the ranks' slabs in rank order -- the same bits on every
  // rank and replica
  char* xr_base[PEER_MAX_RANKS];
  int xr_world, xr_rank;
  unsigned xr_tag0;
  long long xr_timeout;             // its waits' spin limit (ticks): ranks may start seconds apart
  long long o_xt;                   // total slabs [2][wgs][PM_XSLOT] (replica 0's workspace; xr_world > 1)
  // parameter-server hook (V1 roles; async / hogwild frequency='batch', reference
  // elephas/worker.py:114-127): after its update every owning workgroup pushes its
  // delta (theta_new - theta_pulled, fp32 atomics into the sharded device PS) and pulls
  // its slice of theta for the next step, inside the launch.  ps_mode 0 off, 1 hogwild,
  // 2 asynchronous (a pull never sees a half-applied push of a slice: per-slice
  // began / ended counters, slice = the owning workgroup's index, in rank 0's flag area)
  int ps_mode;
  PsArgs ps;
  int bf16;                         // V2 only: X and the weight images are bf16 (mixed_bfloat16 policy)
  // the epilogue also writes both weight-image parities (V2: 0 -- the host marks them stale
  // and rebuilds them from the masters before the next reader; the transposed image's
  // stores are strided)
  int imgs;
  int act0, act1, act2;
  float rate0, rate1;
  int bias0, bias1, bias2;
  long long p_off0, p_off1, p_off2;
  const float* X; long long sX, ldx;
  const float* Y; long long sY, ldy;
  const int* perm; long long sPerm;
  const int* ntrain;
  float* P; long long sP;
  float* S; long long sS;
  OptParams op;
  float* Wsh; long long sWsh, wsh_par;
  float* WTsh; long long sWTsh, wtsh_par;
  long long wsh_off[3], wtsh_off[3];
  int Np[3], Kp[3];
  int loss, nmet, met[4];
  double* acc; int acc_stride;
  long long* ctr;
  unsigned long long seed;
  float* ws; long long ws_stride;   // per-replica exchange workspace (floats)
  long long o_part, o_dz0, o_a0, o_a1, o_dz1, o_dz2, o_w1, o_w2, o_b1, o_b2;
  unsigned* flags;                  // [R][PMF_N][PM_MAXWG], zero at launch (cleared by the chunk's post node)
  unsigned* err;                    // sticky error word (a timed-out wait), read by the host
  long long timeout;                // spin limit in s_memrealtime ticks (100 MHz)
  long long* stamps;                // diagnostics: [block][PM_STAMP_STEPS][32] s_memrealtime (null = off)
  // fused replica averaging at the end of the launch (the reference's fit-end average,
  // spark_model.py:221-227, when the host asks for it right after this chunk): every
  // workgroup's masters reach P write-through, a grid barrier (counter flag_at(0, PMF_AVG)),
  // then workgroup b averages its slice of the avg_n parameters over the R replicas (fp64 in
  // replica order, * avg_scale) into avg_out (if set) and every replica's P (if avg_p)
  int avg_end, avg_p;
  long long avg_n;
  double avg_scale;
  float* avg_out;
};
constexpr int PM_STAMP_STEPS = 8;

// --------------------------------------- persistent layer pipeline (deep.hip)
// A chunk of training steps of a 2..DP_MAXL-layer Dense stack whose hidden layers are too
// wide / too many for PersistArgs (Otto 93-512-512-512-9 at B = 128): nw workgroups per
// replica (512 threads each, one per CU).  Workgroup j OWNS column tile j (16 units) of
// every hidden layer: W_0[:, J] (its forward + weight gradient) and, for layers l >= 1, the
// ROWS J of W_l (the input-gradient stripe dA_{l-1}[:, J] and the weight gradient
// DW_l[J, :] of the backward); the forward of layer l >= 1 reads the columns J of W_l from a
// transposed image the row owners rewrite after their update.  Phases of a step are
// separated by per-replica all-to-all flag barriers (see deep.hip).
constexpr int DP_MAXL = 5;      // Dense layers
constexpr int DP_MAXWG = 64;    // workgroups per replica (one polling wave)
constexpr int DP_MAX_DEVICES = 64;   // devices a process may launch the layer pipeline on
constexpr int DP_ROWS = 128;    // batch rows per replica
constexpr int DP_MAXC = 32;     // last-layer units (whole rows in one loss tile)
constexpr int DP_CW = 64;       // dZ columns per backward chunk
constexpr int DP_STAMP_STEPS = 8;
struct DeepLayer {
  int K, N;            // true input / output widths
  int N16;             // output width padded to 16
  int Kx;              // input row stride (multiple of 8): layer 0 the shard's ldx, else N16 below
  int T;               // 16-column tiles of the output
  int act, has_bias;
  float rate;
  long long p_off;     // kernel [K][N] at p_off of the flat vector, bias (N) after it
  long long o_a, o_dz; // workspace (floats): A_l, dZ_l [Bp][N16] (hidden layers; dZ also last)
  long long o_wt;      // workspace: W_l^T image [N16][Kx] (l >= 1)
  long long o_w;       // workspace: row-major image [Kx][N16] (last layer)
  int l_w;             // LDS: owned master -- layer 0: W^T tile [16][Kx + 4]; l >= 1: rows [16][N16 + 4]
  int l_b;             // LDS: owned bias tile [16] (last layer: [N16] on workgroup 0)
  int l_at;            // LDS: A_l^T stripe [16][Bp + 4] (hidden layers)
};
struct DeepArgs {
  int R, B, Bp, RT, KS, nsteps, L, nw;
  DeepLayer ly[DP_MAXL];
  long long o_g, o_bl;          // workspace: G_{L-2} [Bp][N16], last-layer bias image [N16]
  int l_dz0, l_stage, l_red, lds_floats;
  const float* X; long long sX, ldx;
  const float* Y; long long sY, ldy;
  const int* perm; long long sPerm;
  const int* ntrain;
  float* P; long long sP;
  float* S; long long sS;
  OptParams op;
  int loss, nmet, met[4];
  double* acc; int acc_stride;
  long long* ctr;
  unsigned long long seed;
  float* ws; long long ws_stride;   // per-replica workspace (floats)
  unsigned* flags;                  // [R][4][DP_MAXWG] GO / phase / exchange counters, zero at launch
  // per-step synchronous replicas (sync != 0): every workgroup's weight-gradient tile goes
  // through the exchange buffer xg -- partial tiles [R][nw][XT], then the replica sums
  // [nw][XT]; in a tile, W_0[:, J]^T at 0 ([16][Kx0]), b_0[J] at x_b0, rows J of W_l at
  // x_w[l] ([16][N16_l]) and b_l at x_b[l] (l >= 1)
  int sync, XT, x_b0;
  int x_w[DP_MAXL], x_b[DP_MAXL];
  float* xg;
  // per-step sync across ranks (xr_world > 1): after the replica reduce-scatter, replica r's
  // slice of workgroup j's summed tile goes through every rank's peer-mapped buffer
  // (peer_args.h): data [2 parities][nw][XT] floats at PEER_DATA_OFF, flag (j * R + r) at
  // PEER_FLAG_OFF + 64 (j R + r); tags xr_tag0 + step + 1 (monotonic over the trainer's life)
  char* xr_base[PEER_MAX_RANKS];
  int xr_world, xr_rank;
  unsigned xr_tag0;
  long long xr_timeout;
  // in-launch parameter-server hook (ps_mode 1 hogwild / 2 asynchronous; the kernel then runs
  // its gradient tiles through xg as in sync, without the replica sum): after each step's
  // update every workgroup pushes theta_new - theta_old of the parameters it owns and pulls
  // them for the next step (slice j of the server's per-slice counters)
  int ps_mode;
  PsArgs ps;
  unsigned* err;                    // sticky error word (PmErr codes)
  long long timeout;                // spin limit in s_memrealtime ticks
  long long* stamps;                // diagnostics: [block][DP_STAMP_STEPS][32] s_memrealtime (null = off)
};

constexpr int MAX_SEG = 16;

struct Seg {
  long long p_off;   // offset of the kernel matrix [K][N] in the flat vector
  int K, N;          // kernel shape; bias (if any) follows at p_off + K*N
  int has_bias;
  long long wsh_off, ldwsh;    // row-major shadow W  [K][ldwsh]
  long long wtsh_off, ldwtsh;  // transposed shadow W^T [N][ldwtsh]
};

struct FlatArgs {
  int R;
  long long n;        // params per replica
  float* P; long long sP;
  const float* G; long long sG;
  float* S; long long sS;
  OptParams op;
  int nseg;
  Seg seg[MAX_SEG];
  void* Wsh; long long sWsh, wsh_par;
  void* WTsh; long long sWTsh, wtsh_par;
  long long* ctr;
  const int* ntrain; int B;
  int both_parities;  // refresh: write both shadow parities
  // refresh from an external vector (parameter-server pull): every replica's P and
  // shadows are rebuilt from src; replica 0 also copies src into src_copy
  const float* src; float* src_copy;
  int total_blocks;
};

}  // namespace ea
