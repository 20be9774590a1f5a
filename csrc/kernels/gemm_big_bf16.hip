// Grouped GEMM instantiation: the 256x256 8-wave ping-pong tile (gemm_big.h), bf16,
// one variant per kind set a launch can hold.
#include <cstdlib>

#include "gemm_big.h"

namespace ea {
// the production schedule: V 1 (A half-tiles staged one phase earlier, three half-tiles in
// flight across the k-tile wait). Interleaved A/B with bf16 C (tools/big_ab.py,
// profiles/big_ab_r5.txt), best / median TF: 4096^3 V1 1176 / 1118, V0 1176 / 1102, V5 1151 /
// 1058; 8192^3 1303 / 1284, 1270 / 1266, 1260 / 1250 -- within a few per cent of each other
// (single-order runs, profiles/big_variants_r5.txt, mostly measure clock warm-up)
constexpr int BIG_V = 1;
// tile order of multi-replica launches (gemm_big G): ELEPHAS_AMD_BIG_GROUP=1 groups of 4 tile rows
static int big_group() {
  static const int g = [] {
    const char* e = std::getenv("ELEPHAS_AMD_BIG_GROUP");
    return (e && std::atoi(e) != 0) ? 1 : 0;
  }();
  return g;
}
template <unsigned KM0, unsigned KM1>
static bool big_if(const GroupArgs& ga, hipStream_t s, hipError_t& e) {
  if (!(KM0 & KB(ga.p[0].kind))) return false;
  if (ga.nprob > 1 && !(KM1 & KB(ga.p[1].kind))) return false;
  if (big_group() && ga.R > 1)
    hipLaunchKernelGGL((gemm_big<KM0, KM1, BIG_V, 1>), dim3(ga.R, ga.total_blocks), dim3(BIG_NT), BIG_LDS, s, ga);
  else
    hipLaunchKernelGGL((gemm_big<KM0, KM1, BIG_V>), dim3(ga.R, ga.total_blocks), dim3(BIG_NT), BIG_LDS, s, ga);
  e = hipGetLastError();
  return true;
}
template <unsigned KM0, unsigned KM1, int V = 0, int G = 0> static void big_attr() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big<KM0, KM1, V, G>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, BIG_LDS);
}
constexpr unsigned KM_PLAIN_ = KB(PK_PLAIN);
}  // namespace ea

extern "C" hipError_t ea_gemm_launch_big_bf16(const ea::GroupArgs* ga, hipStream_t s) {
  using namespace ea;
  if (ga->total_blocks <= 0) return hipSuccess;
  hipError_t e = hipSuccess;
  if (big_if<KM_PLAIN_, KM_NONE>(*ga, s, e) || big_if<KM_FWD, KM_NONE>(*ga, s, e) ||
      big_if<KM_DW, KM_DX>(*ga, s, e) || big_if<KM_DX, KM_NONE>(*ga, s, e))
    return e;
  return hipErrorInvalidValue;  // a kind the big tile has no epilogue for (loss, gather, split-K)
}

// schedule variants of the plain GEMM for tools/big_variants.py / big_ab.py: cfg 5 -> V 5,
// 6 -> V 6, 7 -> V 0 (the production cfg 4 runs BIG_V)
extern "C" hipError_t ea_gemm_launch_big_var_bf16(const ea::GroupArgs* ga, int v, hipStream_t s) {
  using namespace ea;
  if (ga->total_blocks <= 0) return hipSuccess;
  if (ga->nprob != 1 || ga->p[0].kind != PK_PLAIN) return hipErrorInvalidValue;
  if (v == 1) hipLaunchKernelGGL((gemm_big<KM_PLAIN_, KM_NONE, 5>), dim3(ga->R, ga->total_blocks), dim3(BIG_NT), BIG_LDS, s, *ga);
  else if (v == 2) hipLaunchKernelGGL((gemm_big<KM_PLAIN_, KM_NONE, 6>), dim3(ga->R, ga->total_blocks), dim3(BIG_NT), BIG_LDS, s, *ga);
  else hipLaunchKernelGGL((gemm_big<KM_PLAIN_, KM_NONE, 0>), dim3(ga->R, ga->total_blocks), dim3(BIG_NT), BIG_LDS, s, *ga);
  return hipGetLastError();
}

extern "C" void ea_gemm_init_big_bf16() {
  using namespace ea;
  big_attr<KM_PLAIN_, KM_NONE, 5>();
  big_attr<KM_PLAIN_, KM_NONE, 6>();
  big_attr<KM_PLAIN_, KM_NONE, 0>();
  big_attr<KM_PLAIN_, KM_NONE, BIG_V>();
  big_attr<KM_FWD, KM_NONE, BIG_V>();
  big_attr<KM_DW, KM_DX, BIG_V>();
  big_attr<KM_DX, KM_NONE, BIG_V>();
  big_attr<KM_PLAIN_, KM_NONE, BIG_V, 1>();
  big_attr<KM_FWD, KM_NONE, BIG_V, 1>();
  big_attr<KM_DW, KM_DX, BIG_V, 1>();
  big_attr<KM_DX, KM_NONE, BIG_V, 1>();
}
