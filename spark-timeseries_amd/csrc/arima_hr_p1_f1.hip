// arima_hr_p1_f1.hip — explicit instantiation of k_hr_init for AR order p = 1, fused differencing on
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(1, true, )
}  // namespace sts
