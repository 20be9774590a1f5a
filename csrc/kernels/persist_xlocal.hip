// Exchange-local instance of the persistent replica-cluster kernel (per-step sync of 8
// replicas on the V1 roles): persist.hip compiled again with EA_PLOCAL = 2 -- the 8 copies of
// every gradient tile on one XCD, the replica-sum exchange kept in that XCD's L2 (see the
// note at the top of persist.hip) -- in a namespace of its own.  Entry: ea_persist_xlocal.
#define EA_PLOCAL 2
#define ea ea_xchglocal
#include "persist.hip"
