// arima_hr_p0_f0.hip — explicit instantiation of k_hr_init for AR order p = 0, fused differencing off
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(0, false, )
}  // namespace sts
