// arima_inst_p5.hip — explicit instantiation of the order-specialised kernels for AR order p = 5
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_P(5, )
}  // namespace sts
