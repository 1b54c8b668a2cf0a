// Multi-GPU row sharding helpers, so that an N-GPU step runs
// no PyTorch compute between its first and last event:
//   dps_shard_edges     work-balanced contiguous row shards from the build's
//                       per-row work terms (device scan + binary search), and
//                       the comparison with a reference plan (no read-back);
//   dps_pack_counts     (count << 32) | index words of a top-k block, the
//                       8-byte wire format of the gather;
//   dps_unpack_gathered rank 0's gathered [world * m, k] words back to
//                       (index, count, score) in row order, the score rebuilt
//                       with the hot kernel's one fp64 division of the same
//                       exact integers (DPathSim_APVPA.py:51-52), so the bits
//                       are identical to the ones the rank computed.
// The reference has no counterpart: its Spark session (:146-168) moves the
// .count() results (:86, :107) back to the driver one target at a time.
#include "dps_common.hpp"

namespace dps {
namespace {

constexpr int kBlock = 256;

// edges[r] (r = 1..world-1) = number of rows i whose inclusive work prefix
// W(i) = pre[i+1] + (i+1) * hm is <= cut_r = r * W(n-1) / world, with
// hm = (sum terms / n) / 2 -- the row work terms + half the mean of
// PathSimEngine.row_work().  W is nondecreasing, so a binary search per cut.
__global__ __launch_bounds__(kBlock) void k_shard_edges(const int64_t* __restrict__ pre, int64_t n,
                                                        int world, int64_t* __restrict__ edges,
                                                        const int64_t* __restrict__ ref,
                                                        int64_t* __restrict__ mismatch) {
  __shared__ int64_t e[kBlock + 1];
  const int r = threadIdx.x;
  const int64_t S = pre[n];
  const int64_t hm = (S / n) / 2;
  const int64_t total = S + n * hm;
  if (r <= world) {
    int64_t v;
    if (r == 0) {
      v = 0;
    } else if (r == world) {
      v = n;
    } else {
      const int64_t cut = static_cast<int64_t>(r) * total / world;
      int64_t lo = 0, hi = n;                     // count of i with W(i) <= cut
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (pre[mid + 1] + (mid + 1) * hm <= cut) lo = mid + 1;
        else hi = mid;
      }
      v = lo;
    }
    e[r] = v;
  }
  __syncthreads();
  if (r == 0) {                                    // running maximum (monotone already)
    int64_t m = 0, bad = 0;
    for (int i = 0; i <= world; ++i) {
      m = e[i] > m ? e[i] : m;
      m = m < n ? m : n;
      edges[i] = m;
      if (ref) bad += ref[i] != m;
    }
    if (ref && mismatch) *mismatch += bad;
  }
}

__global__ __launch_bounds__(kBlock) void k_shard_edges_empty(int world, int64_t* __restrict__ edges,
                                                              const int64_t* __restrict__ ref,
                                                              int64_t* __restrict__ mismatch) {
  if (threadIdx.x != 0) return;
  int64_t bad = 0;
  for (int i = 0; i <= world; ++i) {
    edges[i] = 0;
    if (ref) bad += ref[i] != 0;
  }
  if (ref && mismatch) *mismatch += bad;
}

__global__ __launch_bounds__(kBlock) void k_pack_counts(const int32_t* __restrict__ idx,
                                                        const int64_t* __restrict__ cnt, int64_t n,
                                                        int64_t* __restrict__ out) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    out[i] = static_cast<int64_t>((static_cast<uint64_t>(cnt[i]) << 32) |
                                  static_cast<uint32_t>(idx[i]));
}

// One thread per output slot: row x = edges[0] + i / k lives in the shard r
// with edges[r] <= x < edges[r+1], at gathered row r * m + (x - edges[r]).
__global__ __launch_bounds__(kBlock) void k_unpack_gathered(const int64_t* __restrict__ gathered,
                                                            int world, int64_t m, int k,
                                                            int64_t n_rows,
                                                            const int64_t* __restrict__ edges,
                                                            const int64_t* __restrict__ den,
                                                            int32_t* __restrict__ out_idx,
                                                            int64_t* __restrict__ out_cnt,
                                                            double* __restrict__ out_score) {
  const int64_t x0 = edges[0];
  // the out_* arrays hold n_rows rows: never more, whatever the device edges say
  const int64_t span = edges[world] - x0;
  const int64_t n = (span < n_rows ? span : n_rows) * k;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t x = x0 + i / k;
    const int s = static_cast<int>(i % k);
    int r = 0;
    while (r + 1 < world && edges[r + 1] <= x) ++r;
    if (x - edges[r] >= m) continue;   // a shard longer than the gathered block: not sent
    const uint64_t w = static_cast<uint64_t>(gathered[(r * m + (x - edges[r])) * k + s]);
    const int32_t y = static_cast<int32_t>(static_cast<uint32_t>(w));
    const int64_t c = static_cast<int64_t>(w >> 32);
    double sc = 0.0;
    if (y >= 0 && c > 0)
      sc = static_cast<double>(2 * c) / static_cast<double>(den[x] + den[y]);
    out_idx[i] = y;
    out_cnt[i] = c;
    out_score[i] = sc;
  }
}

}  // namespace
}  // namespace dps

using namespace dps;

extern "C" {

size_t dps_shard_edges_workspace_size(int64_t n_rows) {
  if (n_rows < 0) return 0;
  return align_up(static_cast<size_t>(n_rows + 1) * sizeof(int64_t)) + scan_workspace_size(n_rows) +
         256;
}

int dps_shard_edges(const int64_t* terms, int64_t n_rows, int32_t world, int64_t* edges,
                    const int64_t* edges_ref, int64_t* mismatch, void* ws, size_t ws_bytes,
                    void* stream) {
  DPS_REQUIRE(world >= 1 && world <= kBlock - 1, DPS_ERR_INVALID, "world must be in [1, %d], got %d",
              kBlock - 1, world);
  DPS_REQUIRE(n_rows >= 0, DPS_ERR_INVALID, "bad n_rows");
  DPS_REQUIRE(edges, DPS_ERR_INVALID, "null edges");
  DPS_REQUIRE(!edges_ref || mismatch, DPS_ERR_INVALID, "edges_ref needs a mismatch counter");
  auto st = static_cast<hipStream_t>(stream);
  if (n_rows == 0) {
    k_shard_edges_empty<<<1, kBlock, 0, st>>>(world, edges, edges_ref, mismatch);
    DPS_LAUNCHED();
    return DPS_OK;
  }
  DPS_REQUIRE(terms, DPS_ERR_INVALID, "null terms");
  Carve cv(ws, ws_bytes);
  int64_t* pre = cv.take<int64_t>(static_cast<size_t>(n_rows + 1));
  const size_t sb = scan_workspace_size(n_rows);
  void* sws = cv.take<char>(sb);
  DPS_REQUIRE(cv.ok, DPS_ERR_WORKSPACE, "workspace too small (%zu bytes)", ws_bytes);
  DPS_HIP_RET(scan_exclusive<int64_t>(terms, pre, n_rows, sws, sb, st));
  k_shard_edges<<<1, kBlock, 0, st>>>(pre, n_rows, world, edges, edges_ref, mismatch);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_pack_counts(const int32_t* idx, const int64_t* cnt, int64_t n, int64_t* out, void* stream) {
  DPS_REQUIRE(n >= 0, DPS_ERR_INVALID, "bad n");
  if (n == 0) return DPS_OK;
  DPS_REQUIRE(idx && cnt && out, DPS_ERR_INVALID, "null array");
  k_pack_counts<<<grid_for(n, kBlock), kBlock, 0, static_cast<hipStream_t>(stream)>>>(idx, cnt, n, out);
  DPS_LAUNCHED();
  return DPS_OK;
}

int dps_unpack_gathered(const int64_t* gathered, int32_t world, int64_t m, int32_t k,
                        const int64_t* edges, int64_t n_rows, const int64_t* den, int32_t* out_idx,
                        int64_t* out_cnt, double* out_score, void* stream) {
  DPS_REQUIRE(world >= 1, DPS_ERR_INVALID, "bad world %d", world);
  DPS_REQUIRE(k >= 1 && m >= 0 && n_rows >= 0, DPS_ERR_INVALID, "bad k / m / n_rows");
  if (n_rows == 0) return DPS_OK;
  DPS_REQUIRE(gathered && edges && den && out_idx && out_cnt && out_score, DPS_ERR_INVALID,
              "null array");
  k_unpack_gathered<<<grid_for(n_rows * k, kBlock), kBlock, 0, static_cast<hipStream_t>(stream)>>>(
      gathered, world, m, k, n_rows, edges, den, out_idx, out_cnt, out_score);
  DPS_LAUNCHED();
  return DPS_OK;
}

}  // extern "C"
