// Row-window conv kernels with 32-output-channel tiles (conv_win.h), one
// translation unit per tile width so the build compiles them in parallel.
#define UNET_WIN_IMPL
#include "conv_win.h"

namespace unet {
template hipError_t launch_win<32, 512>(const ConvFwdParams&, hipStream_t);
template hipError_t launch_win<32, 256>(const ConvFwdParams&, hipStream_t);
}  // namespace unet
