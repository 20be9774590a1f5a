// Grouped GEMM instantiation: 128x64 THR-N64 tile, bf16.
// One tile config per translation unit so the configs compile in parallel.
#include "gemm_impl.h"

extern "C" hipError_t ea_gemm_launch_thr64_bf16(const ea::GroupArgs* ga, hipStream_t s) {
  return ea::launch_cfg<__bf16, 4, 2, 2, 2, 1, true>(*ga, s);
}

extern "C" hipError_t ea_gemm_dual_bf16(const ea::GroupArgs* ga, int a, int b, hipStream_t s) {
  return ea::launch_dual<__bf16>(*ga, a, b, s);
}

extern "C" void ea_gemm_init_thr64_bf16() {
  using namespace ea;
  set_attr_spec<__bf16, 4, 2, 2, 2, 1>();
  set_attr_dual<__bf16>();
}
