// Register-resident fast path (K=7 / K=9).  Placeholder until the kernel lands.
#include "vtb_internal.h"

namespace vtb {

bool reg_path_supported(const Launch&) { return false; }

hipError_t launch_reg_path(const Launch&) { return hipErrorNotSupported; }

}  // namespace vtb
