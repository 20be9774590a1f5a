// Launch-argument structs shared by the device kernels and the native executor
// (csrc/runtime/executor.cpp). Plain-old-data only: passed by value as kernel args.
#pragma once
#include <stdint.h>

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
  PK_LOSS_ROWS = 7   // wide final layer: one wave per row over fp32 logits Z
};

struct Prob {
  int kind;
  int M, N, K;             // K: padded reduction length (multiple of 8)
  int R;                   // replicas
  int tiles_m, tiles_n;
  int block_begin;
  // operands
  const void* A; long long lda, sA;
  const void* BT; long long ldb, sB;
  int a_gather;            // 1: A rows come from the batch window (train: perm, eval: contiguous)
  int a_rowstep;           // with a_gather: the epoch's rows are pre-permuted, batch row m = step * B + m
  int a_colstep;           // A advances by step * B elements per step (pre-permuted X^T of layer 0)
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
  int total_blocks;
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
  float* Bsh; long long sBsh, bsh_par;  // fp32 bias images per parity (fused tail only), flat index
  long long* ctr;
  const int* ntrain; int B;
  int both_parities;  // refresh: write both shadow parities
  // refresh from an external vector (parameter-server pull): every replica's P and
  // shadows are rebuilt from src; replica 0 also copies src into src_copy
  const float* src; float* src_copy;
  int total_blocks;
};

// ------------------------------------------------------------ fused MLP tail
// One workgroup per replica runs, for layers 1..L-1 of a small MLP, the
// forward pass, the loss, and the backward pass with every weight update, with
// all activations resident in LDS (see fused.hip). Layer 0's forward (wide K)
// and weight update (many tiles) stay on the grouped GEMM kernel.
constexpr int FUSED_MAX_L = 8;

struct FusedLayer {
  int K, N, Kp, Np;        // dims; Kp/Np padded to 8
  int act, has_bias;
  float rate;
  int ldA;                 // LDS row stride (elements) of this layer's output D_l / dZ_l tiles
  int offD;                // LDS byte offset of D_l (compute dtype, [64][ldA]) (l < L-1)
  int offG;                // LDS byte offset of G_l (fp32 [64][ldG]): z, then act'(z)*dropout (l < L-1)
  int ldG;
  int pvec;                // P/S rows of this layer allow float4 access (N % 4 == 0, p_off % 4 == 0)
  long long p_off;         // flat parameter offset (kernel K*N, then bias N)
  long long wsh_off, wtsh_off;
};

struct FusedArgs {
  int L;
  int nsplit;              // workgroups per replica (each owns 1/nsplit of the update tiles)
  const FusedLayer* ly;    // device array [L] (uniform loads)
  int R, B, Bp;
  // layer-0 outputs of the grouped forward launch
  const void* D0; long long sD0;   // [B][Np0] compute dtype
  const float* Z0; long long sZ0;  // [B][N0]  fp32
  // targets
  const float* Y; long long sY, ldy;
  const int* perm; long long sPerm;
  const int* ntrain;
  // out: dZ_0^T [N0][Bp] (B^T operand of the layer-0 weight update)
  void* dZ0T; long long sdZ0T;
  // deferred layer-1 update (nsplit == 1 mode): the tail writes dZ_1^T [N1][Bp]
  // and skips layer 1's weight update, which runs with layer 0's in the next
  // grouped launch; nullptr = the tail updates every layer >= 1 itself
  void* dZ1T; long long sdZ1T;
  // parameters
  float* P; long long sP;
  float* S; long long sS;
  OptParams op;
  void* Wsh; long long sWsh, wsh_par;
  void* WTsh; long long sWTsh, wtsh_par;
  // fp32 bias images per parity, indexed like P: the forward of layer l reads the
  // current parity while other workgroups of the replica write the next one
  float* Bsh; long long sBsh, bsh_par;
  int loss, nmet, met[4];
  double* acc; int acc_stride;
  long long* ctr; int step_off;
  unsigned long long seed;
  // LDS layout
  int offLg, ldLg;         // logits / dZ_{L-1} fp32 [64][ldLg]
  int offdZ0, offdZ1;      // dZ ping-pong (compute dtype [64][lddZ])
  int lddZ;
  int offY, offSrow;       // targets fp32 [64][32], row flags int[64]
  int lds_bytes;
  long long* stamps;
};

}  // namespace ea
