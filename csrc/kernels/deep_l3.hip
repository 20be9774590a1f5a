// Instances of the persistent layer-pipeline kernel for 3 Dense layers (deep_impl.h)
#include "deep_impl.h"

extern "C" hipError_t ea_deep_l3(const ea::DeepArgs* a, int fast, int opk, hipStream_t s) {
  return ea::deep_launch<3>(a, fast != 0, opk, s);
}
