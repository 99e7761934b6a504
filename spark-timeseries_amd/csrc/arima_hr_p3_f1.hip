// arima_hr_p3_f1.hip — explicit instantiation of k_hr_init for AR order p = 3, fused differencing on
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(3, true, )
}  // namespace sts
