// Diagnostic (not product): does K1's XCD-contiguous tile walk lose HBM bandwidth for some chunk
// sizes?  A pure streaming read with the scan's geometry: tiles of 256 rows x 1536 B (384 KiB),
// 8 x 32 persistent walkers (blockIdx & 7 = XCD group), each XCD group owning a contiguous range of
// the chunk's tiles, walker w of a group reading tiles lo + w, lo + w + 32, ...  Walk variants:
//   0 contiguous (as shipped)   1 contiguous, each XCD's walk rotated by x/8 of its range
//   2 interleaved (tile t on XCD group t & 7)
// Prints GB/s per (rows, variant) over a 15.4 GB buffer (10M rows), reading rows [r0, r0 + rows).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/diag/hbm_camp.hip -o tools/diag/hbm_camp
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int ROWB = 1536, TROWS = 256;
constexpr int64_t TILEB = (int64_t)ROWB * TROWS;

__global__ __launch_bounds__(512) void walk(const uint8_t* __restrict__ base, int64_t tiles, int var,
                                            unsigned* __restrict__ out) {
  const int xcd = blockIdx.x & 7, w = blockIdx.x >> 3, G = gridDim.x >> 3;
  const int64_t q = tiles >> 3, rem = tiles & 7;
  const int64_t lo = xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
  const int64_t cnt = q + (xcd < rem ? 1 : 0);
  u4 acc = {0u, 0u, 0u, 0u};
  for (int64_t i = w; i < (var == 2 ? (tiles + 7 - xcd) / 8 : cnt); i += G) {
    int64_t t;
    if (var == 2)
      t = i * 8 + xcd;
    else if (var == 1)
      t = lo + (i + cnt * xcd / 8) % cnt;
    else
      t = lo + i;
    const u4* p = reinterpret_cast<const u4*>(base + t * TILEB);
#pragma unroll 4
    for (int j = threadIdx.x; j < (int)(TILEB / 16); j += 512) acc ^= p[j];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

int main() {
  const int64_t N = 10000000;
  uint8_t* buf;
  unsigned* out;
  (void)hipMalloc(&buf, N * ROWB);
  (void)hipMalloc(&out, 4);
  (void)hipMemset(buf, 1, N * ROWB);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int64_t cases[][2] = {{598016, 4194304}, {4792320, 5207680}, {0, 4194304}, {598016, 3300000},
                              {0, 2097152}, {0, 1048576}, {598016, 4194304 + 256 * 8 * 3}};
  for (auto& c : cases) {
    const int64_t tiles = c[1] / TROWS;
    for (int var = 0; var < 3; ++var) {
      const uint8_t* b = buf + c[0] * ROWB;
      hipLaunchKernelGGL(walk, dim3(256), dim3(512), 0, 0, b, tiles, var, out);
      (void)hipEventRecord(e0);
      const int reps = 5;
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(walk, dim3(256), dim3(512), 0, 0, b, tiles, var, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double gbs = (double)tiles * TILEB * reps / (ms * 1e-3) / 1e9;
      printf("r0 %8lld rows %8lld tiles/xcd %6lld var %d: %7.1f GB/s  (%.3f ms per pass)\n", (long long)c[0],
             (long long)c[1], (long long)(tiles / 8), var, gbs, ms / reps);
      fflush(stdout);
    }
  }
  return 0;
}
