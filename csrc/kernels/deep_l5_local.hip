// XCD-local instances of the persistent layer-pipeline kernel for 5 Dense layers (deep_impl.h
// with EA_DLOCAL = 1, in a namespace of its own; fit granularity)
#define EA_DLOCAL 1
#define ea ea_dlocal
#include "deep_impl.h"

extern "C" hipError_t ea_deep_l5_local(const ea::DeepArgs* a, int fast, int opk, hipStream_t s) {
  return ea::deep_launch<5>(a, fast != 0, opk, s);
}
