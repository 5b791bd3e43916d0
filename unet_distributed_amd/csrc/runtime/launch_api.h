// Host-side entry points of the HIP kernels (implemented in csrc/kernels/*.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include "../kernels/conv_params.h"

namespace unet {

const char* conv_fwd_prepare(ConvFwdParams& p);
hipError_t conv_fwd_launch(const ConvFwdParams& p, hipStream_t s);

const char* wgrad_check(const WgradParams& p);
WgradCfg wgrad_pick(const WgradParams& p);
hipError_t wgrad_launch(const WgradParams& p, hipStream_t s);
hipError_t wgrad_reduce_launch(const float* slab, int splits, int taps, int Mtot, int Mout, int Nc, int rg, int rkeep,
                               float scale, float* out, float* stage, hipStream_t s);
size_t wgrad_reduce_stage_floats(int splits, int taps, int Mtot, int Nc);
int reduce_groups(int splits);
hipError_t multi_reduce_launch(const void* jobs, int njobs, long long total1, long long total2, hipStream_t s);
hipError_t colsum_launch(const void* x, int rows, int C, int blocks, float* partial, hipStream_t s);

hipError_t cast_input_launch(const float* x, int P, int Cin, int Cpad, void* y, hipStream_t s);
hipError_t maxpool2_fwd_launch(const void* x, int N, int D, int H, int W, int C, int dims3, void* y, hipStream_t s);
hipError_t maxpool2_bwd_launch(const void* x, const void* dy, const void* skip, int N, int D, int H, int W, int C,
                               int dims3, void* dx, hipStream_t s);
hipError_t upsample2_bwd_launch(const void* dup, const void* mask, int N, int D, int H, int W, int C, int dims3,
                                void* dlow, hipStream_t s);

int head_blocks(int P);
const char* head_check(int C);
hipError_t head_fwd_launch(const void* x, const float* w, const float* b, const void* t, int P, int C, float* prob,
                           float* partial, float* sums, hipStream_t s);
hipError_t head_bwd_launch(const void* x, const float* w, const float* prob, const void* t, const float* sums, int P,
                           int C, float inv_total, float bce_w, float gscale, void* dx, float* partial, float* gw,
                           float* gb, hipStream_t s);
hipError_t partial_reduce_launch(const float* partial, int nb, int width, float* out, hipStream_t s);

int norm_blocks_per_sample(int N, int P);
const char* norm_check(int C, int G);
hipError_t norm_moments_launch(const void* A, const void* B, int N, int P, int C, float* partial, float* S,
                               hipStream_t s);
hipError_t bn_finalize_launch(const float* S, int N, int C, float count, int mode, const float* gamma, float eps,
                              float momentum, float* run_mean, float* run_var, float* mean, float* rstd, float* ca,
                              float* cb, float* cc, float* dgamma, float* dbeta, hipStream_t s);
hipError_t gn_finalize_launch(const float* S, int N, int C, int G, int P, int mode, const float* gamma, float eps,
                              float* mean, float* rstd, float* ca, float* cb, float* cc, float* dgamma, float* dbeta,
                              hipStream_t s);
hipError_t norm_apply_launch(const void* z, int N, int P, int C, const float* mean, const float* rstd, int cstride,
                             const float* gamma, const float* beta, int relu, float drop_rate, uint32_t seed,
                             const uint32_t* seed_ptr, uint32_t salt, void* y, hipStream_t s);
hipError_t norm_bwd_apply_launch(const void* g, const void* z, int N, int P, int C, const float* ca, const float* cb,
                                 const float* cc, int cstride, void* dz, hipStream_t s);

const char* adam_check(int nseg);
hipError_t adam_pack_launch(float* w, const float* g, float* m, float* v, int n_total, const void* segs, int nseg,
                            float lr_t, float b1, float b2, float eps, float gscale, int do_adam,
                            const float* dev_scalars, void* arena, hipStream_t s);

uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n);
void gather_rows(const uint8_t* src, const int64_t* idx, int64_t n, int64_t row_bytes, uint8_t* dst, int threads);

}  // namespace unet
