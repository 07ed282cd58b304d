/* kfmi_inst_ac128_k2.hip -- kernel instantiations for K=2, LAY_AC128 (see kfmi_kernels.h). */
#include "kfmi_kernels.h"

namespace kfmi {
KFMI_FOR_NB(KFMI_INSTANTIATE, 2, LAY_AC128)
}  // namespace kfmi
