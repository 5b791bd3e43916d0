// Pipelined 8-wave row-window conv (conv_pipe.h) in its own translation unit so the
// build compiles it in parallel with the other window variants.
#define UNET_PIPE_IMPL
#include "conv_pipe.h"
