/* kfmi_inst_grp_k4.hip -- kernel instantiations for K=4, d=64, LAY_GRP (see kfmi_kernels.h). */
#include "kfmi_kernels.h"

namespace kfmi {
KFMI_INSTANTIATE(4, 2, LAY_GRP)
}  // namespace kfmi
