// Host-check build only (tests/test_host_sanitizers.py): the shape-validation binary links
// conv_fwd.hip's host code, which dispatches to the row-window launchers of
// conv_win_b{32,64}.hip.  It never launches a kernel, so these stand-ins keep the
// sanitizer build from compiling ~150 gfx950 kernel variants it would not run.
#include "conv_win.h"

namespace unet_types {
bool dry_dispatch() { return false; }
}  // namespace unet_types

namespace unet {
template <int BN, int BM>
hipError_t launch_win(const ConvFwdParams&, hipStream_t) {
  return hipErrorNotSupported;
}
template hipError_t launch_win<32, 512>(const ConvFwdParams&, hipStream_t);
template hipError_t launch_win<32, 256>(const ConvFwdParams&, hipStream_t);
template hipError_t launch_win<64, 256>(const ConvFwdParams&, hipStream_t);
const char* conv_dw_check(const ConvFwdParams& p) {
  return p.fw.x ? "host-check build: no fused weight-gradient kernel" : nullptr;
}
int conv_dw_grid(const ConvFwdParams& p) { return p.fw.nsplit; }
int conv_dw_stat_rows(const ConvFwdParams& p) { return p.N * p.OH / 2; }
hipError_t launch_conv_dw(const ConvFwdParams&, hipStream_t) { return hipErrorNotSupported; }
}  // namespace unet
