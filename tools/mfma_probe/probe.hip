// MFMA probe (research tool, not product code): how fast can the heavy-venue
// part of C.C^T run on gfx950 i8 MFMA?  M_H = P . P^T for a dense i8 panel P
// [targets x K] (K heaviest venues, targets in label order), sources = the
// first n_src labels, with the minimal per-element epilogue a hybrid kernel
// needs: a light-term bound read from LDS, the max of every lane's 16 results
// and a compare against the source's threshold (candidates counted).
//
// Shape: 256 threads = 4 waves; a block owns 128 sources (32 per wave, held as
// the MFMA B operand in registers) and sweeps every target in tiles of 256
// (A operand, double-buffered in LDS, 8 blocks of 32 targets), K/32
// v_mfma_i32_32x32x32_i8 per 32x32 block.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kTT = 256;    // targets per tile

template <int K>
__global__ __launch_bounds__(256) void k_probe(const int8_t* __restrict__ panel, int64_t n_t,
                                               const int32_t* __restrict__ thr, int64_t n_src,
                                               unsigned long long* __restrict__ cnt,
                                               int32_t* __restrict__ dump) {
  // 256 sources per block: wave w owns sources [64w, 64w+64) as two 32-column
  // B sets, so every A fragment read from LDS feeds two MFMAs; A rows are
  // padded to K+16 bytes (no bank conflicts across the 32 rows of a fragment)
  constexpr int KS = K / 32;                 // k-slices
  constexpr int RS = K + 16;                 // LDS row stride (bytes)
  __shared__ __attribute__((aligned(16))) int8_t a_s[2][kTT * RS];
  __shared__ uint32_t light_s[1024];         // 4 KB stand-in for the light terms
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t src0 = static_cast<int64_t>(blockIdx.x) * 256 + wave * 64;
  for (int i = tid; i < 1024; i += 256) light_s[i] = 0;
  v4i b[2][KS];
  int th[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int64_t s = src0 + 32 * c + r;
    const int64_t sr = s < n_src ? s : 0;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      b[c][ks] = *reinterpret_cast<const v4i*>(panel + sr * K + 32 * ks + 16 * h);
    th[c] = s < n_src ? thr[s] : 0x7FFFFFFF;
  }
  const int64_t n_tiles = (n_t + kTT - 1) / kTT;
  auto stage = [&](int buf, int64_t t) {
    const int8_t* src = panel + t * kTT * K;
    const int64_t rows = min<int64_t>(kTT, n_t - t * kTT);
    for (int i = tid; i < kTT * (K / 16); i += 256) {
      const int row = i / (K / 16), part = i % (K / 16);
      v4i v = {0, 0, 0, 0};
      if (row < rows) v = *reinterpret_cast<const v4i*>(src + row * K + part * 16);
      *reinterpret_cast<v4i*>(&a_s[buf][row * RS + part * 16]) = v;
    }
  };
  stage(0, 0);
  __syncthreads();
  unsigned long long found = 0;
  for (int64_t t = 0; t < n_tiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < n_tiles) stage(buf ^ 1, t + 1);
#pragma unroll 2
    for (int blk = 0; blk < kTT / 32; ++blk) {
      v16i acc[2] = {{}, {}};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const v4i a = *reinterpret_cast<const v4i*>(&a_s[buf][(blk * 32 + r) * RS + 32 * ks + 16 * h]);
        acc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b[0][ks], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b[1][ks], acc[1], 0, 0, 0);
      }
      if (dump && blockIdx.x == 0 && t == 0 && wave < 2) {   // verification
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int row = (g & 3) + 8 * (g >> 2) + 4 * h;   // target within the block
          dump[(wave * 64 + r) * 256 + blk * 32 + row] = acc[0][g];
        }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint32_t* lp = light_s + ((r + 32 * c) * 16 + blk * 4) % 1024;
        const uint32_t lor = lp[0] | lp[1] | lp[2] | lp[3];
        const int lb = static_cast<int>(max(max(lor & 0xFF, (lor >> 8) & 0xFF),
                                            max((lor >> 16) & 0xFF, lor >> 24)));
        const v16i& x = acc[c];
        int m0 = max(max(x[0], x[1]), x[2]);
        int m1 = max(max(x[3], x[4]), x[5]);
        int m2 = max(max(x[6], x[7]), x[8]);
        int m3 = max(max(x[9], x[10]), x[11]);
        int m4 = max(max(x[12], x[13]), x[14]);
        int mx = max(max(max(m0, m1), max(m2, m3)), max(m4, x[15]));
        if (mx + lb >= th[c]) ++found;
      }
    }
    __syncthreads();
  }
  if (found) atomicAdd(cnt, found);
}

extern "C" int probe_run(const int8_t* panel, int64_t n_t, int K, const int32_t* thr,
                         int64_t n_src, unsigned long long* cnt, int32_t* dump, void* stream) {
  const unsigned grid = static_cast<unsigned>((n_src + 255) / 256);
  auto st = static_cast<hipStream_t>(stream);
  if (K == 64) k_probe<64><<<grid, 256, 0, st>>>(panel, n_t, thr, n_src, cnt, dump);
  else if (K == 128) k_probe<128><<<grid, 256, 0, st>>>(panel, n_t, thr, n_src, cnt, dump);
  else if (K == 32) k_probe<32><<<grid, 256, 0, st>>>(panel, n_t, thr, n_src, cnt, dump);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
