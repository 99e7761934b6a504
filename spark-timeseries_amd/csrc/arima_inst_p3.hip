// arima_inst_p3.hip — explicit instantiation of the order-specialised kernels for AR order p = 3
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_P(3, )
}  // namespace sts
