// pm_fitch_nt.hip -- the Fitch passes of pm_fitch.hip with non-temporal set-record loads
// (PM_NT_LOADS, see load_rec in pm_kernels.h): launch_fitch_nt, the launch sequence a run
// whose levels are large takes (nt_policy in pm_host.cpp).
#define PM_NT_LOADS 1
#include "pm_fitch.hip"
