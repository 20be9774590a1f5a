// Instances of the persistent layer-pipeline kernel for 2 Dense layers (deep_impl.h)
#define EA_DEEP_XRANK_ENTRY 1   // the rank-exchange self-test entry lives in this unit
#include "deep_impl.h"

extern "C" hipError_t ea_deep_l2(const ea::DeepArgs* a, int fast, int opk, hipStream_t s) {
  return ea::deep_launch<2>(a, fast != 0, opk, s);
}
