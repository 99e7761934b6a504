// arima_cg_p4_s0.hip — explicit instantiation of the fit kernel (k_cg_fit) for AR order p = 4, Breeze
// reading smear = 0 (its own translation unit: the heaviest kernel, so the build parallelises over it)
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_CG(4, false, )
}  // namespace sts
