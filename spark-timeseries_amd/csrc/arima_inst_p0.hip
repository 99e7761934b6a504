// arima_inst_p0.hip — explicit instantiation of the order-specialised kernels for AR order p = 0
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_P(0, )
}  // namespace sts
