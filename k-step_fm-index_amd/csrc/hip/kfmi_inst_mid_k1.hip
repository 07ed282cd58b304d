/* kfmi_inst_mid_k1.hip -- kernel instantiations for K=1, LAY_MID (see kfmi_kernels.h). */
#include "kfmi_kernels.h"

namespace kfmi {
KFMI_FOR_NB(KFMI_INSTANTIATE, 1, LAY_MID)
}  // namespace kfmi
