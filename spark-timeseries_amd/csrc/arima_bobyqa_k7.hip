// css-bobyqa kernels of dimension 7 (arima_bobyqa_impl.hpp), one translation unit per dimension
#include "arima_bobyqa_impl.hpp"

namespace sts {
STS_BQ_DECLARE(7, )
}  // namespace sts
