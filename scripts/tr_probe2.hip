#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s4 __attribute__((ext_vector_type(4)));
template <int NB> __device__ int trswz(int k) {
  if constexpr (NB == 2) return (k >> 3) & 1;
  if constexpr (NB == 4) return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
  if constexpr (NB >= 8) return (k & 3) | (((k >> 3) & 1) << 2);
  return 0;
}
template <int W> __device__ int tr_off(int k, int c) {
  constexpr int NB = W / 16;
  return k * W * 2 + (((c >> 4) ^ trswz<NB>(k)) << 5) + ((c & 15) << 1);
}
template <int W>
__global__ void probe(short* out, int cbase) {
  __shared__ __attribute__((aligned(16))) char smem[32 * W * 2];
  for (int i = threadIdx.x; i < 32 * W; i += 64) {
    int k = i / W, c = i % W;
    *(short*)(smem + tr_off<W>(k, c)) = (short)(k * 100 + c);
  }
  __syncthreads();
  const char* img = smem;
  int lane = threadIdx.x;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(img + tr_off<W>(8 * g + q, cbase + 4 * pp)));
  s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(img + tr_off<W>(8 * g + 4 + q, cbase + 4 * pp)));
  for (int j = 0; j < 4; ++j) { out[lane * 8 + j] = lo[j]; out[lane * 8 + 4 + j] = hi[j]; }
}
int main() {
  short* d; (void)hipMalloc(&d, 64 * 8 * 2);
  short h[512];
  for (int cb : {0, 16}) {
    probe<32><<<1, 64>>>(d, cb);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("W=32 cbase=%d\n", cb);
    for (int l = 0; l < 64; l += 5) { printf("lane %2d:", l); for (int j = 0; j < 8; ++j) printf(" %5d", h[l * 8 + j]); printf("\n"); }
  }
  probe<128><<<1, 64>>>(d, 32);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("W=128 cbase=32\n");
  for (int l = 0; l < 64; l += 5) { printf("lane %2d:", l); for (int j = 0; j < 8; ++j) printf(" %5d", h[l * 8 + j]); printf("\n"); }
  return 0;
}
