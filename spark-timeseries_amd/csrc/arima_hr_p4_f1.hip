// arima_hr_p4_f1.hip — explicit instantiation of k_hr_init for AR order p = 4, fused differencing on
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_HR(4, true, )
}  // namespace sts
