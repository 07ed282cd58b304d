/* kfmi_inst_inter_k2.hip -- kernel instantiations for K=2, LAY_INTER (see kfmi_kernels.h). */
#include "kfmi_kernels.h"

namespace kfmi {
KFMI_FOR_NB(KFMI_INSTANTIATE, 2, LAY_INTER)
}  // namespace kfmi
