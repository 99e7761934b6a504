// arima_cg_p0_s1.hip — explicit instantiation of the fit kernel (k_cg_fit) for AR order p = 0, Breeze
// reading smear = 1 (its own translation unit: the heaviest kernel, so the build parallelises over it)
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_CG(0, true, )
}  // namespace sts
