// arima_hr_p2_f0.hip — explicit instantiation of k_hr_init for AR order p = 2, fused differencing off
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(2, false, )
}  // namespace sts
