// Grouped GEMM instantiation: 64x64 split-K-2 tile, bf16.
// One tile config per translation unit so the configs compile in parallel.
#include "gemm_impl.h"

extern "C" hipError_t ea_gemm_launch_lat64_bf16(const ea::GroupArgs* ga, hipStream_t s) {
  return ea::launch_cfg<__bf16, 4, 2, 1, 2, 2>(*ga, s);
}

extern "C" void ea_gemm_init_lat64_bf16() {
  using namespace ea;
  set_attr<__bf16, 4, 2, 1, 2, 2>();
}
