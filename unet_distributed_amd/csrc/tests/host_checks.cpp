// Host-side checks of the native runtime under the sanitizers: built by
// tests/test_host_sanitizers.py with g++ -fsanitize=address,undefined and, separately,
// -fsanitize=thread (the multi-threaded row gather of the data loader is the runtime's
// only host concurrency).  GPU AddressSanitizer / xnack+ runs are not available on the
// MI355X pool, so device code is covered by the GPU numerics tests instead.
//
// With -DUNET_WITH_SHAPE_CHECKS the launch-shape validation of conv_fwd.hip /
// conv_wgrad.hip (host code compiled by hipcc, `-Xarch_host -fsanitize=...`) is swept
// over the UNet level shapes and a set of invalid shapes as well.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

namespace unet {
uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n);
void gather_rows(const uint8_t* src, const int64_t* idx, int64_t n, int64_t row_bytes, uint8_t* dst, int threads);
}  // namespace unet

#ifdef UNET_WITH_SHAPE_CHECKS
#include "launch_api.h"
#endif

static int failures = 0;
#define CHECK(cond)                                                  \
  do {                                                               \
    if (!(cond)) {                                                   \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                    \
    }                                                                \
  } while (0)

static void check_crc32c() {
  const char* s = "123456789";
  CHECK(unet::crc32c_extend(0, (const uint8_t*)s, 9) == 0xE3069283u);
  std::mt19937 rng(1);
  std::vector<uint8_t> buf(4099);
  for (auto& b : buf) b = (uint8_t)rng();
  for (size_t off = 0; off < 9; ++off) {          // unaligned starts, every tail length
    const uint8_t* p = buf.data() + off;
    const size_t n = buf.size() - off;
    const uint32_t whole = unet::crc32c_extend(0, p, n);
    for (size_t cut : {size_t(0), size_t(1), size_t(7), size_t(8), n / 3, n - 1, n}) {
      const uint32_t part = unet::crc32c_extend(unet::crc32c_extend(0, p, cut), p + cut, n - cut);
      CHECK(part == whole);
    }
  }
}

static void check_gather() {
  std::mt19937 rng(2);
  for (int64_t row_bytes : {int64_t(1), int64_t(12), int64_t(4096 + 3)}) {
    for (int64_t n : {int64_t(0), int64_t(1), int64_t(63), int64_t(64), int64_t(1000)}) {
      const int64_t rows = 257;
      std::vector<uint8_t> src(rows * row_bytes);
      for (auto& b : src) b = (uint8_t)rng();
      std::vector<int64_t> idx(n);
      for (auto& i : idx) i = (int64_t)(rng() % rows);
      std::vector<uint8_t> ref(n * row_bytes + 1, 0xAB);
      for (int64_t i = 0; i < n; ++i) memcpy(ref.data() + i * row_bytes, src.data() + idx[i] * row_bytes, row_bytes);
      for (int threads : {0, 1, 3, 8, 64}) {
        std::vector<uint8_t> dst(n * row_bytes + 1, 0xAB);   // guard byte must survive
        unet::gather_rows(src.data(), idx.data(), n, row_bytes, dst.data(), threads);
        CHECK(dst == ref);
      }
    }
  }
}

#ifdef UNET_WITH_SHAPE_CHECKS
static void check_shapes() {
  using unet_types::ConvFwdParams;
  int ok = 0, rejected = 0;
  for (int img : {8, 16, 32, 64, 128, 256, 512})
    for (int cin : {4, 8, 32, 48, 64, 128, 512})
      for (int c2 : {0, 32, 64})
        for (int cout : {32, 40, 64, 512}) {
          ConvFwdParams p{};
          p.N = 2; p.OD = p.ID = 1; p.OH = p.OW = p.IH = p.IW = img;
          p.KD = 1; p.KH = p.KW = 3; p.stride = 1; p.pad = 1;
          p.C1 = cin; p.C2 = c2; p.up1 = 1; p.Cout = cout; p.D1 = cout; p.relu = 1; p.out_scale = 1.f;
          p.src1 = (const void*)16; p.src2 = c2 ? (const void*)16 : nullptr; p.wgt = (const void*)16;
          p.dst1 = (void*)16; p.mask_scale1 = p.mask_scale2 = 1.f;
          if (unet::conv_fwd_prepare(p) == nullptr) {
            ++ok;
            CHECK(p.Kpad % 64 == 0 && p.Kpad >= 9 * (cin + c2));
            CHECK(unet::conv_fwd_grid(p) >= 0);
          } else {
            ++rejected;
          }
        }
  CHECK(ok > 0 && rejected > 0);
}
#endif

int main() {
  check_crc32c();
  check_gather();
#ifdef UNET_WITH_SHAPE_CHECKS
  check_shapes();
#endif
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("host checks passed\n");
  return 0;
}
