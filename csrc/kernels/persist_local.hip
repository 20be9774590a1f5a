// XCD-local instance of the persistent replica-cluster kernel: persist.hip compiled again
// with EA_PLOCAL = 1 (intra-replica hand-offs kept in the XCD's L2; see the note at the top
// of persist.hip), in a namespace of its own so that no template instance of the two
// builds can stand in for the other at link time.  Entry point: ea_persist_local.
#define EA_PLOCAL 1
#define ea ea_xcdlocal
#include "persist.hip"
