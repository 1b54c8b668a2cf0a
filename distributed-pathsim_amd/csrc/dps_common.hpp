// Shared helpers for libdpathsim (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstddef>
#include <cstdint>

#include "dps_host.hpp"

namespace dps {

constexpr int kWave = 64;

// Target tiles of the C^T layout (dps_tiles.hip, dps_cct1.hip): W = 2^shift
// labels for shift in [8, 16], or the T15 layout -- 15 / 16 of 8192 / 16384,
// i.e. 7680 (u8 entries, shift 13) or 15360 (4-bit entries, shift 14), whose
// 7680-byte accumulator keeps 20 one-wave workgroups resident on a CU (8 KiB
// keeps 18, Geo in dps_cct1.hip).  Labels are < 2^31.
struct TileDim {
  int shift;   // entry format; log2(W) unless t15
  bool t15;
  __host__ __device__ int64_t w() const {
    return t15 ? int64_t(15) << (shift - 4) : int64_t(1) << shift;
  }
  __host__ __device__ int64_t tile(int64_t lab) const {
    return t15 ? static_cast<int64_t>(static_cast<uint32_t>(lab >> (shift - 4)) / 15u) : lab >> shift;
  }
  __host__ __device__ uint32_t local(int64_t lab) const {
    return static_cast<uint32_t>(lab - tile(lab) * w());
  }
};
// The tile width's TileDim; shift = -1 when the width is not one of them.
inline TileDim tile_dim(int32_t w) {
  if (w == 7680) return TileDim{13, true};
  if (w == 15360) return TileDim{14, true};
  int s = 0;
  while (s < 31 && (1 << s) < w) ++s;
  return TileDim{(1 << s) == w && s >= 8 && s <= 16 ? s : -1, false};
}

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// Bump allocator over the caller's workspace (never allocates device memory).
struct Carve {
  char* base;
  size_t cap;
  size_t off = 0;
  bool ok = true;
  Carve(void* p, size_t n) : base(static_cast<char*>(p)), cap(n) {}
  template <class T>
  T* take(size_t count) {
    size_t bytes = align_up(count * sizeof(T));
    if (off + bytes > cap) { ok = false; return nullptr; }
    T* p = reinterpret_cast<T*>(base + off);
    off += bytes;
    return p;
  }
};

inline int grid_for(int64_t n, int block, int64_t cap = 2048 * 4) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

// ---- wave64 primitives ------------------------------------------------------
__device__ __forceinline__ int lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// number of set bits of `mask` strictly below this lane
__device__ __forceinline__ int mbcnt(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(mask), 0u));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ unsigned readlane(unsigned v, int l) {
  return static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}
__device__ __forceinline__ int64_t readlane(int64_t v, int l) {
  int lo = __builtin_amdgcn_readlane(static_cast<int>(static_cast<uint64_t>(v)), l);
  int hi = __builtin_amdgcn_readlane(static_cast<int>(static_cast<uint64_t>(v) >> 32), l);
  return static_cast<int64_t>((static_cast<uint64_t>(static_cast<unsigned>(hi)) << 32) |
                              static_cast<unsigned>(lo));
}
// int64 of a per-lane source lane (ds_bpermute x 2; readlane needs a uniform lane)
__device__ __forceinline__ int64_t readlane_var(int64_t v, int src) {
  const uint64_t u = static_cast<uint64_t>(v);
  const unsigned lo = static_cast<unsigned>(__shfl(static_cast<int>(u), src, kWave));
  const unsigned hi = static_cast<unsigned>(__shfl(static_cast<int>(u >> 32), src, kWave));
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}
__device__ __forceinline__ double readlane(double v, int l) {
  return __longlong_as_double(readlane(static_cast<int64_t>(__double_as_longlong(v)), l));
}

template <class T>
__device__ __forceinline__ T wave_inclusive_sum(T v) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    T t = __shfl_up(v, d, kWave);
    if (lane >= d) v += t;
  }
  return v;
}
template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}
template <class T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    T o = __shfl_xor(v, d, kWave);
    v = o > v ? o : v;
  }
  return v;
}

template <class T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    T o = __shfl_xor(v, d, kWave);
    v = o < v ? o : v;
  }
  return v;
}

// atomicMax on a hot device-wide address, skipped when a (possibly stale, but
// monotone) read already shows a value >= v: a few record-breaking updates
// instead of one serialised atomic per wave.
__device__ __forceinline__ void atomic_max_filtered(unsigned long long* p, unsigned long long v) {
  if (v > __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(p, v);
}

// Flattened iteration over 64 lane-held segments: with `excl` the exclusive
// prefix of the segment lengths (non-decreasing over lanes), the segment that
// owns flattened entry i is the largest lane j with excl_j <= i (empty
// segments are skipped because the next lane has the same prefix).
__device__ __forceinline__ int wave_owner(uint32_t excl, uint32_t i) {
  int j = 0;
#pragma unroll
  for (int step = kWave / 2; step > 0; step >>= 1) {
    const uint32_t e = static_cast<uint32_t>(__shfl(static_cast<int>(excl), j + step, kWave));
    if (e <= i) j += step;
  }
  return j;
}

// Compaction of segmented-unique heads into CSR arrays, for the 64
// consecutive segments s0 .. s0+63: their outputs are one contiguous range
// from out_ptr[s0], walked in coalesced 64-entry strips, each lane finding its
// segment by wave_owner (a lane per segment with a wave for long ones left a
// serial copy loop per lane: config4 296 us).  Every lane must call it.
__device__ __forceinline__ void compact_heads_wave(const int32_t* __restrict__ tmp,
                                                   const int32_t* __restrict__ tmp_cnt,
                                                   const int64_t* __restrict__ seg_ptr,
                                                   const int64_t* __restrict__ out_ptr,
                                                   int64_t n_seg, int32_t* __restrict__ col,
                                                   int32_t* __restrict__ val, int64_t s0) {
  const int lane = lane_id();
  const int64_t sl = s0 + lane;
  const int64_t se = sl < n_seg ? sl : n_seg;
  const int64_t o0 = out_ptr[s0];
  const uint32_t excl = static_cast<uint32_t>(out_ptr[se] - o0);
  const uint32_t total =
      static_cast<uint32_t>(out_ptr[s0 + kWave < n_seg ? s0 + kWave : n_seg] - o0);
  const int64_t src = sl < n_seg ? seg_ptr[sl] : 0;
  for (uint32_t e0 = 0; e0 < total; e0 += kWave) {
    const uint32_t i = e0 + static_cast<uint32_t>(lane);
    const int o = wave_owner(excl, i);
    const int64_t so = readlane_var(src, o);
    const uint32_t eo = static_cast<uint32_t>(__shfl(static_cast<int>(excl), o, kWave));
    if (i < total) {
      const int64_t j = so + (i - eo);
      col[o0 + i] = tmp[j];
      if (val) val[o0 + i] = tmp_cnt[j];
    }
  }
}

// Ascending bitonic sort of one int per lane across the wave.  `lane` is the
// caller's lane id; a kernel that sorts inside a long-lived loop passes it
// through opaque_lane() so that the 21 lane masks of the network are rebuilt
// per call instead of being hoisted out of the loop into 42 SGPRs.
__device__ __forceinline__ int wave_bitonic_sort(int v, int lane) {
#pragma unroll
  for (int k = 2; k <= kWave; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      // partner lane's value by ds_bpermute from `lane` (not __shfl_xor, whose
      // lane-constant addresses the compiler would also hoist)
      int o = __builtin_amdgcn_ds_bpermute((lane ^ j) << 2, v);
      bool up = (lane & k) == 0;
      bool lower = (lane & j) == 0;
      int mn = o < v ? o : v;
      int mx = o < v ? v : o;
      v = (lower == up) ? mn : mx;
    }
  }
  return v;
}
__device__ __forceinline__ int wave_bitonic_sort(int v) { return wave_bitonic_sort(v, lane_id()); }

// The lane id as a value the compiler cannot prove loop-invariant: what is
// derived from it is recomputed where it is used (see wave_bitonic_sort).
__device__ __forceinline__ int opaque_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}

// ---- several dword ranges set in one launch (dps_scan.hip) ---------------------
// Replaces a hipMemsetAsync per small array (each one a fill kernel of its own).
struct FillSet {
  static constexpr int kMax = 16;
  uint32_t* p[kMax];
  int64_t n[kMax];    // dwords
  uint32_t v[kMax];
  int k = 0;
  bool overflow = false;   // an add() beyond kMax ranges (fill_set refuses to run)
  void add(void* ptr, int64_t n_words, uint32_t value) {
    if (k >= kMax) { overflow = true; return; }
    p[k] = static_cast<uint32_t*>(ptr);
    n[k] = n_words;
    v[k] = value;
    ++k;
  }
};
hipError_t fill_set(const FillSet& s, hipStream_t stream);

// ---- device-wide scans (dps_scan.hip) ------------------------------------------
// out[0..n] = exclusive prefix sums of in[0..n), out[n] = total.  ws from
// scan_workspace_size(n).  T in {int32_t, uint32_t, int64_t}.
size_t scan_workspace_size(int64_t n);
template <class T>
hipError_t scan_exclusive(const T* in, int64_t* out, int64_t n, void* ws, size_t ws_bytes,
                          hipStream_t stream);

// ---- segmented sort + unique (+ run counts) (dps_csr.hip) ----------------------
// For every segment s: data[seg_ptr[s] .. seg_ptr[s+1]) is sorted ascending and
// compacted in place to its distinct values (first uniq[s] slots); when
// `counts` is non-null counts[seg_ptr[s] + i] = multiplicity of value i.
// With a SegSrc map the input value at j is map[col[j]] (the single-mid
// SpGEMM's paper -> mid gather, fused into the sort's loads) and data is
// output only.
struct SegSrc {
  const int32_t* col = nullptr;
  const int32_t* map = nullptr;
};
__device__ __forceinline__ int32_t seg_in(const int32_t* data, const SegSrc& src, int64_t j) {
  return src.map ? src.map[src.col[j]] : data[j];
}
size_t seg_unique_workspace_size(int64_t n_seg);
hipError_t seg_unique(int32_t* data, int32_t* counts, const int64_t* seg_ptr, int64_t n_seg,
                      int64_t* uniq, void* ws, size_t ws_bytes, hipStream_t stream,
                      int key_range = 0, SegSrc src = SegSrc());

// ---- stable LSD radix sort of (u64 key, u32 value) pairs (dps_sort.hip) ------
// Sorts by the low key_bits bits of the keys; vals_in == nullptr means values
// 0..n-1.  Outputs must not alias inputs.
size_t radix_sort_workspace_size(int64_t n);
hipError_t radix_sort_pairs(const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out,
                            uint32_t* vals_out, int64_t n, int key_bits, void* ws,
                            size_t ws_bytes, hipStream_t stream);

}  // namespace dps

#define DPS_HIP_RET(call)                                                              \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      dps::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #call,                \
                     hipGetErrorString(e_));                                           \
      return DPS_ERR_HIP;                                                              \
    }                                                                                  \
  } while (0)

#define DPS_LAUNCHED() DPS_HIP_RET(hipGetLastError())

// Device asserts of the debug build (make debug: -DDPS_DEBUG): a failed check
// traps the wave (the launch then reports an error); compiled out otherwise.
#ifdef DPS_DEBUG
#define DPS_DASSERT(cond)                                                              \
  do {                                                                                 \
    if (!(cond)) __builtin_trap();                                                     \
  } while (0)
#else
#define DPS_DASSERT(cond) \
  do {                    \
  } while (0)
#endif
