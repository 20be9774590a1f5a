// Grouped GEMM dispatch: picks the tile-config translation unit (gemm_cfg*.hip,
// gemm_f32.hip) for a launch and runs the wide-output loss rows kernel, which
// is not a GEMM (kernel templates: gemm_impl.h).
#include "gemm_impl.h"

extern "C" {
hipError_t ea_gemm_launch_lat_bf16(const ea::GroupArgs* ga, hipStream_t s);
hipError_t ea_gemm_launch_thr_bf16(const ea::GroupArgs* ga, hipStream_t s);
hipError_t ea_gemm_launch_thr64_bf16(const ea::GroupArgs* ga, hipStream_t s);
hipError_t ea_gemm_launch_lat64_bf16(const ea::GroupArgs* ga, hipStream_t s);
hipError_t ea_gemm_launch_f32(const ea::GroupArgs* ga, int cfg, hipStream_t s);
void ea_gemm_init_lat_bf16();
void ea_gemm_init_thr_bf16();
void ea_gemm_init_thr64_bf16();
void ea_gemm_init_lat64_bf16();
void ea_gemm_init_f32();
}

// cfg: 0 = LAT (64x32, split-K 4), 1 = THR (128x128), 2 = THR-N64 (128x64: twice the
// workgroups for grids that would otherwise leave CUs with a single workgroup),
// 3 = LAT-64 (64x64, 2 N-waves x split-K 2: shallow reductions such as K = batch 64,
// where split-K 4 leaves two waves without a 32-deep chunk)
extern "C" hipError_t ea_gemm_grouped(const ea::GroupArgs* ga, int bf16, int cfg, hipStream_t s) {
  using namespace ea;
  if (ga->total_blocks <= 0) return hipSuccess;
  if (ga->nprob == 1 && ga->p[0].kind == PK_LOSS_ROWS) {
    // dZ^T stage (bf16, LOSS_RPB rows) + the 4-wave x 6 partial-sum reduction
    const size_t lds = (size_t)(LOSS_RPB * LOSS_LDS_MAX_N * 2 + 15) / 16 * 16 + 32 * sizeof(float);
    if (bf16)
      hipLaunchKernelGGL(loss_rows_kernel<__bf16>, dim3(ga->total_blocks), dim3(256), lds, s, *ga);
    else
      hipLaunchKernelGGL(loss_rows_kernel<float>, dim3(ga->total_blocks), dim3(256), lds, s, *ga);
    return hipGetLastError();
  }
  if (!bf16) return ea_gemm_launch_f32(ga, cfg, s);
  if (cfg == 0) return ea_gemm_launch_lat_bf16(ga, s);
  if (cfg == 2) return ea_gemm_launch_thr64_bf16(ga, s);
  if (cfg == 3) return ea_gemm_launch_lat64_bf16(ga, s);
  return ea_gemm_launch_thr_bf16(ga, s);
}

extern "C" void ea_gemm_init() {
  static bool done = false;
  if (done) return;
  ea_gemm_init_lat_bf16();
  ea_gemm_init_thr_bf16();
  ea_gemm_init_thr64_bf16();
  ea_gemm_init_lat64_bf16();
  ea_gemm_init_f32();
  done = true;
}

extern "C" int ea_gemm_tile_m(int cfg) { return (cfg == 0 || cfg == 3) ? 64 : 128; }
extern "C" int ea_gemm_tile_n(int cfg) { return cfg == 0 ? 32 : ((cfg == 2 || cfg == 3) ? 64 : 128); }
extern "C" int ea_gather_tile() { return 64; }
