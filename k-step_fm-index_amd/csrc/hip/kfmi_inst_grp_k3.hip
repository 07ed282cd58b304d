/* kfmi_inst_grp_k3.hip -- kernel instantiations for K=3, d=64, LAY_GRP (see kfmi_kernels.h). */
#include "kfmi_kernels.h"

namespace kfmi {
KFMI_INSTANTIATE(3, 2, LAY_GRP)
}  // namespace kfmi
