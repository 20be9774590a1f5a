// Grouped GEMM instantiation: 64x32 LAT tile, bf16 (plus the kind-specialised variants).
// One tile config per translation unit so the configs compile in parallel.
#include "gemm_impl.h"

extern "C" hipError_t ea_gemm_launch_lat_bf16(const ea::GroupArgs* ga, hipStream_t s) {
  return ea::launch_cfg<__bf16, 4, 2, 1, 1, 4, true>(*ga, s);
}

extern "C" hipError_t ea_gemm_table_lat_bf16(const ea::TableArgs* ta, int dw, hipStream_t s) {
  return ea::launch_table<__bf16>(*ta, dw, s);
}

extern "C" void ea_gemm_init_lat_bf16() {
  using namespace ea;
  set_attr_spec<__bf16, 4, 2, 1, 1, 4>();
  set_attr_table<__bf16>();
}
