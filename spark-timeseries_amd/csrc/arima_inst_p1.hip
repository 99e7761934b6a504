// arima_inst_p1.hip — explicit instantiation of the order-specialised kernels for AR order p = 1
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_P(1, )
}  // namespace sts
