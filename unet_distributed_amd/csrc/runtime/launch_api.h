// Host-side entry points of the HIP kernels (implemented in csrc/kernels/*.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include "../kernels/conv_params.h"

namespace unet {
using namespace unet_types;
#include "launch_api.inc"
}  // namespace unet

namespace unet_f16 {
using namespace unet_types;
#include "launch_api.inc"
}  // namespace unet_f16
