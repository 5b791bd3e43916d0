// Host-side IO helpers of the native runtime (no GPU code):
//  * CRC32C (Castagnoli) with the SSE4.2 crc32 instruction -- used by the TF
//    V2 tensor-bundle checkpoint writer/reader (BundleEntryProto.crc32c, SSTable
//    block trailers) and by the TFRecord framing of TensorBoard event files,
//    matching the formats TF 1.4 wrote for the reference (`test_dist.py:269-271`
//    Saver, `test_dist.py:347-355` Supervisor summaries).
//  * gather_rows: multi-threaded gather of sample rows (with per-epoch
//    permutation) from a memory-mapped .npy into a pinned host batch buffer,
//    the native data-loader primitive behind unet_distributed_amd.data.loader.
#include <nmmintrin.h>
#include <stdint.h>
#include <string.h>

#include <thread>
#include <vector>

namespace unet {

__attribute__((target("sse4.2"))) uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}

// dst[i, :] = src[idx[i], :] for rows of `row_bytes`, split over `threads` host threads.
void gather_rows(const uint8_t* src, const int64_t* idx, int64_t n, int64_t row_bytes, uint8_t* dst, int threads) {
  if (threads < 1) threads = 1;
  if (n < 64) threads = 1;
  std::vector<std::thread> pool;
  const int64_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t b = t * per, e = std::min<int64_t>(n, b + per);
    if (b >= e) break;
    pool.emplace_back([=]() {
      for (int64_t i = b; i < e; ++i) memcpy(dst + i * row_bytes, src + idx[i] * row_bytes, (size_t)row_bytes);
    });
  }
  for (auto& th : pool) th.join();
}

}  // namespace unet
