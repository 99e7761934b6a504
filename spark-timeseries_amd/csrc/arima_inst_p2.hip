// arima_inst_p2.hip — explicit instantiation of the order-specialised kernels for AR order p = 2
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_P(2, )
}  // namespace sts
