/* kfmi_inst_midac_k1.hip -- kernel instantiations for K=1, LAY_MIDAC (see kfmi_kernels.h). */
#include "kfmi_kernels.h"

namespace kfmi {
KFMI_FOR_NB(KFMI_INSTANTIATE, 1, LAY_MIDAC)
}  // namespace kfmi
