// Grouped GEMM instantiations for the fp32 compute policy (exact-f32 MFMA), all
// three tile configs.
#include "gemm_impl.h"

extern "C" hipError_t ea_gemm_launch_f32(const ea::GroupArgs* ga, int cfg, hipStream_t s) {
  using namespace ea;
  if (cfg == 0) return launch_cfg<float, 4, 2, 1, 1, 4>(*ga, s);
  if (cfg == 2) return launch_cfg<float, 4, 2, 2, 2, 1>(*ga, s);
  return launch_cfg<float, 4, 4, 2, 2, 1>(*ga, s);
}

extern "C" hipError_t ea_gemm_dual_f32(const ea::GroupArgs* ga, int a, int b, hipStream_t s) {
  return ea::launch_dual<float>(*ga, a, b, s);
}

extern "C" hipError_t ea_gemm_table_f32(const ea::TableArgs* ta, int dw, hipStream_t s) {
  return ea::launch_table<float>(*ta, dw, s);
}

extern "C" void ea_gemm_init_f32() {
  using namespace ea;
  set_attr_table<float>();
  set_attr_dual<float>();
  set_attr<float, 4, 2, 1, 1, 4>();
  set_attr<float, 4, 4, 2, 2, 1>();
  set_attr<float, 4, 2, 2, 2, 1>();
}
