// pm_sankoff_nt.hip -- the Sankoff passes of pm_sankoff.hip with non-temporal set-record
// loads (PM_NT_LOADS, see load_rec in pm_kernels.h): launch_sankoff_nt, the launch sequence a
// run whose levels are large takes (nt_policy in pm_host.cpp).
#define PM_NT_LOADS 1
#include "pm_sankoff.hip"
