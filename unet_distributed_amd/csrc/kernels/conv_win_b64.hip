// Row-window conv kernels with 64-output-channel tiles (conv_win.h), one
// translation unit per tile width so the build compiles them in parallel.
#define UNET_WIN_IMPL
#include "conv_win.h"

namespace unet {
template hipError_t launch_win<64, 256>(const ConvFwdParams&, hipStream_t);
}  // namespace unet
