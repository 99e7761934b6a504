// arima_inst_p4.hip — explicit instantiation of the order-specialised kernels for AR order p = 4
#include "arima_kernels_impl.hpp"

namespace sts {
STS_DECLARE_P(4, )
}  // namespace sts
