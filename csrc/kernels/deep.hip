// Dispatch of the persistent layer-pipeline kernel (deep_impl.h) to its per-layer-count
// instances (deep_l{2,3,4,5}.hip: one translation unit each, built in parallel)
#include "args.h"
#include <hip/hip_runtime.h>

extern "C" hipError_t ea_deep_l2(const ea::DeepArgs* a, int fast, int opk, hipStream_t s);
extern "C" hipError_t ea_deep_l3(const ea::DeepArgs* a, int fast, int opk, hipStream_t s);
extern "C" hipError_t ea_deep_l4(const ea::DeepArgs* a, int fast, int opk, hipStream_t s);
extern "C" hipError_t ea_deep_l5(const ea::DeepArgs* a, int fast, int opk, hipStream_t s);
extern "C" hipError_t ea_deep_l2_local(const ea::DeepArgs* a, int fast, int opk, hipStream_t s);
extern "C" hipError_t ea_deep_l3_local(const ea::DeepArgs* a, int fast, int opk, hipStream_t s);
extern "C" hipError_t ea_deep_l4_local(const ea::DeepArgs* a, int fast, int opk, hipStream_t s);
extern "C" hipError_t ea_deep_l5_local(const ea::DeepArgs* a, int fast, int opk, hipStream_t s);

using namespace ea;

// grid: R * nw workgroups of 512 threads, every one resident (the host sizes the grid to
// at most one workgroup per CU); dynamic LDS a->lds_floats floats
// local != 0: the XCD-local instances (deep_l*_local.hip; the host checked R % 8 == 0, fit)
extern "C" hipError_t ea_deep(const DeepArgs* a, int local, hipStream_t s) {
  if (a->nsteps <= 0) return hipSuccess;
  // softmax + (sparse) categorical cross-entropy with accuracy / CCE metrics: the quad-per-row
  // loss tile; everything else the generic one
  bool fast = a->ly[a->L - 1].act == ACT_SOFTMAX && (a->loss == LOSS_CCE || a->loss == LOSS_SPARSE_CCE);
  for (int i = 0; i < a->nmet; ++i)
    fast = fast && (a->met[i] == MET_ACC_CAT || a->met[i] == MET_ACC_SPARSE || a->met[i] == LOSS_CCE ||
                    a->met[i] == LOSS_SPARSE_CCE);
  // the kernel's optimizer instance: 0 plain SGD (no optimizer state), 1 Adam, 2 any other
  // rule (run-time dispatch) -- deep_impl.h OPK_*
  const int opk = (a->op.opt == OPT_SGD && a->op.mom == 0.f) ? 0 : (a->op.opt == OPT_ADAM ? 1 : 2);
  switch (a->L) {
    case 2: return local ? ea_deep_l2_local(a, fast, opk, s) : ea_deep_l2(a, fast, opk, s);
    case 3: return local ? ea_deep_l3_local(a, fast, opk, s) : ea_deep_l3(a, fast, opk, s);
    case 4: return local ? ea_deep_l4_local(a, fast, opk, s) : ea_deep_l4(a, fast, opk, s);
    case 5: return local ? ea_deep_l5_local(a, fast, opk, s) : ea_deep_l5(a, fast, opk, s);
    default: return hipErrorInvalidValue;
  }
}
