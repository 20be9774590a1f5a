// Grouped GEMM dispatch: picks the tile-config translation unit (gemm_cfg*.hip,
// gemm_f32.hip) for a launch and runs the wide-output loss rows kernel, which
// is not a GEMM (kernel templates: gemm_impl.h).
#include <mutex>

#include "gemm_impl.h"

extern "C" {
hipError_t ea_gemm_launch_lat_bf16(const ea::GroupArgs* ga, hipStream_t s);
hipError_t ea_gemm_launch_thr_bf16(const ea::GroupArgs* ga, hipStream_t s);
hipError_t ea_gemm_launch_thr64_bf16(const ea::GroupArgs* ga, hipStream_t s);
hipError_t ea_gemm_launch_big_bf16(const ea::GroupArgs* ga, hipStream_t s);
hipError_t ea_gemm_launch_big_var_bf16(const ea::GroupArgs* ga, int v, hipStream_t s);
hipError_t ea_gemm_launch_f32(const ea::GroupArgs* ga, int cfg, hipStream_t s);
hipError_t ea_gemm_dual_f32(const ea::GroupArgs* ga, int a, int b, hipStream_t s);
hipError_t ea_gemm_dual_bf16(const ea::GroupArgs* ga, int a, int b, hipStream_t s);
hipError_t ea_gemm_table_lat_bf16(const ea::TableArgs* ta, int dw, hipStream_t s);
hipError_t ea_gemm_table_f32(const ea::TableArgs* ta, int dw, hipStream_t s);
void ea_gemm_init_lat_bf16();
void ea_gemm_init_thr_bf16();
void ea_gemm_init_thr64_bf16();
void ea_gemm_init_big_bf16();
void ea_gemm_init_f32();
}

// cfg: 0 = LAT (64x32, split-K 4), 1 = THR (128x128), 2 = THR-N64 (128x64: twice the
// workgroups for grids that would otherwise leave CUs with a single workgroup),
// 4 = BIG (256x256, 8 ping-pong waves, bf16 only: gemm_big.h)
extern "C" hipError_t ea_gemm_grouped(const ea::GroupArgs* ga, int bf16, int cfg, hipStream_t s) {
  using namespace ea;
  if (ga->total_blocks <= 0) return hipSuccess;
  if (ga->nprob == 1 && ga->p[0].kind == PK_LOSS_ROWS) {
    // dZ^T stage (bf16, LOSS_RPB rows) + the 4-wave x 6 partial-sum reduction
    const size_t lds = (size_t)(LOSS_RPB * LOSS_LDS_MAX_N * 2 + 15) / 16 * 16 + 32 * sizeof(float);
    if (bf16)
      hipLaunchKernelGGL(loss_rows_kernel<__bf16>, dim3(ga->R, ga->total_blocks), dim3(256), lds, s, *ga);
    else
      hipLaunchKernelGGL(loss_rows_kernel<float>, dim3(ga->R, ga->total_blocks), dim3(256), lds, s, *ga);
    return hipGetLastError();
  }
  // 100 + 10 a + b: problem 0 on config a, problem 1 on config b (gemm_dual)
  if (cfg >= 100) return bf16 ? ea_gemm_dual_bf16(ga, (cfg - 100) / 10, cfg % 10, s)
                              : ea_gemm_dual_f32(ga, (cfg - 100) / 10, cfg % 10, s);
  if (!bf16) return ea_gemm_launch_f32(ga, cfg >= 4 ? 1 : cfg, s);
  if (cfg == 4) return ea_gemm_launch_big_bf16(ga, s);
  if (cfg >= 5) return ea_gemm_launch_big_var_bf16(ga, cfg - 4, s);
  if (cfg == 0) return ea_gemm_launch_lat_bf16(ga, s);
  if (cfg == 2) return ea_gemm_launch_thr64_bf16(ga, s);
  return ea_gemm_launch_thr_bf16(ga, s);
}

// row-chain plan table launches: dw = 0 -> {layer-0 split-K partial, X^T gather}
// on the 64x32 LAT tile; dw = 1 -> {DW of every layer} on a 64x64 tile
extern "C" hipError_t ea_gemm_table(const ea::TableArgs* ta, int bf16, int dw, hipStream_t s) {
  return bf16 ? ea_gemm_table_lat_bf16(ta, dw, s) : ea_gemm_table_f32(ta, dw, s);
}

// the function attributes (dynamic-LDS limits) are per device: raised once on each device a
// process builds an executor on, under a lock (executors may be built from several threads)
extern "C" void ea_gemm_init() {
  static std::mutex mu;
  static bool done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  std::lock_guard<std::mutex> g(mu);
  if (done[dev]) return;
  ea_gemm_init_lat_bf16();
  ea_gemm_init_thr_bf16();
  ea_gemm_init_thr64_bf16();
  ea_gemm_init_big_bf16();
  ea_gemm_init_f32();
  done[dev] = true;
}

// cfg 3: the 64x64 tile of the row-chain weight-gradient table launch (not a
// grouped-launch config)
// (a dual config 100 + 10 a + b reports its first problem's tile)
extern "C" int ea_gemm_tile_m(int cfg) {
  if (cfg >= 100) cfg = (cfg - 100) / 10;
  return cfg >= 4 ? 256 : ((cfg == 0 || cfg == 3) ? 64 : 128);
}
extern "C" int ea_gemm_tile_n(int cfg) {
  if (cfg >= 100) cfg = (cfg - 100) / 10;
  return cfg >= 4 ? 256 : (cfg == 0 ? 32 : ((cfg == 2 || cfg == 3) ? 64 : 128));
}
extern "C" int ea_gather_tile() { return 64; }
