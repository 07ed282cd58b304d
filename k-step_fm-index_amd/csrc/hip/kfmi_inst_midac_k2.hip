/* kfmi_inst_midac_k2.hip -- kernel instantiations for K=2, LAY_MIDAC (see kfmi_kernels.h). */
#include "kfmi_kernels.h"

namespace kfmi {
KFMI_FOR_NB(KFMI_INSTANTIATE, 2, LAY_MIDAC)
}  // namespace kfmi
