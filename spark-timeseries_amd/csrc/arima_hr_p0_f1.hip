// arima_hr_p0_f1.hip — explicit instantiation of k_hr_init for AR order p = 0, fused differencing on
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(0, true, )
}  // namespace sts
