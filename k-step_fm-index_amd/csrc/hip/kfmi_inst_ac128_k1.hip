/* kfmi_inst_ac128_k1.hip -- kernel instantiations for K=1, LAY_AC128 (see kfmi_kernels.h). */
#include "kfmi_kernels.h"

namespace kfmi {
KFMI_FOR_NB(KFMI_INSTANTIATE, 1, LAY_AC128)
}  // namespace kfmi
