// Probe the lane semantics of ds_read_b64_tr_b16 on gfx950: LDS[r][c] = r*100 + c (16-bit),
// every lane supplies address of (row = lane-derived, col block), dump what each lane receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s4 __attribute__((ext_vector_type(4)));
__global__ void probe(short* out, int mode) {
  __shared__ short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = (short)((i / 64) * 100 + (i % 64));
  __syncthreads();
  int lane = threadIdx.x;
  int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  int row = 8 * g + q, col = 4 * p;           // my assumed addressing
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(lds + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[lane * 4 + j] = v[j];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  probe<<<1, 64>>>(d, 0);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) { printf("lane %2d:", l); for (int j = 0; j < 4; ++j) printf(" %5d", h[l * 4 + j]); printf("\n"); }
  return 0;
}
