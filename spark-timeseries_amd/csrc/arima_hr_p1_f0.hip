// arima_hr_p1_f0.hip — explicit instantiation of k_hr_init for AR order p = 1, fused differencing off
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(1, false, )
}  // namespace sts
