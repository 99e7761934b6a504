// arima_hr_p5_f0.hip — explicit instantiation of k_hr_init for AR order p = 5, fused differencing off
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(5, false, )
}  // namespace sts
