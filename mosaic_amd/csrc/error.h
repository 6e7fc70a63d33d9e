// Status + thread-local message of the C ABI (mgpu_last_error), for every
// translation unit of libmosaic_gpu.so (defined in capi.cpp).
#pragma once
#include <stdint.h>

namespace mgpu {
int32_t set_error(int32_t code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}
