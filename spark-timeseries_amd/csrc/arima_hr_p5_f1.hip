// arima_hr_p5_f1.hip — explicit instantiation of k_hr_init for AR order p = 5, fused differencing on
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(5, true, )
}  // namespace sts
