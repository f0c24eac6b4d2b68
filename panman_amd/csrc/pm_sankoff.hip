// pm_sankoff.hip -- placeholder until the Sankoff kernels land: the product fails loudly.
#include "pm_internal.h"

namespace pm {
hipError_t launch_sankoff(pm_ctx*) { return hipErrorNotSupported; }
}  // namespace pm
