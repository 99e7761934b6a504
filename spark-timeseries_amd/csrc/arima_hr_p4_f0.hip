// arima_hr_p4_f0.hip — explicit instantiation of k_hr_init for AR order p = 4, fused differencing off
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(4, false, )
}  // namespace sts
