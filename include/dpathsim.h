/*
 * dpathsim.h -- C ABI of libdpathsim.so, the MI355X (gfx950) PathSim engine.
 *
 * This is the drop-in boundary for the reference's hot path.
 * The reference (phamtheanhphu/Distributed-PathSim, DPathSim_APVPA.py) has no
 * FFI: its "operator API" is a graphframes motif query + Spark SQL filters +
 * distinct().count() called from the Python class DPathSim_APVPA.  Each entry
 * point below names the reference element it replaces (file:line into
 * /root/reference).  The Python host package (dpathsim, ctypes) mirrors the
 * reference class on top of these; INTEGRATION.md shows the bindings.
 *
 * Conventions
 *  - Every function returns int status: 0 = DPS_OK, < 0 = error code; the
 *    message is in dps_last_error() (thread-local).  No C++ exception crosses
 *    the ABI.
 *  - All array pointers are DEVICE pointers (allocated by the caller, e.g. as
 *    PyTorch-ROCm tensors) unless the parameter name ends in _host.
 *  - Work is enqueued asynchronously on the caller's hipStream_t `stream`
 *    (passed as void*; NULL = the legacy default stream).  Outputs are valid
 *    after the stream is synchronised.  No function allocates device memory
 *    or synchronises the stream, except where documented ("syncs").
 *  - Scratch comes from a caller workspace `ws` of `ws_bytes` bytes; the
 *    matching *_workspace_size() gives the required size.  `ws` must be
 *    256-byte aligned.
 *  - Not re-entrant per stream; one host thread may drive several devices
 *    (call hipSetDevice / pass that device's stream).
 *
 * Index spaces (built host-side from node types only, see dpathsim/graph.py):
 *  - node n in [0, N_nodes): GEXF node order (DPathSim_APVPA.py:120-121).
 *  - node_rowid[n]: author-typed nodes get [0, N_A) in node order, every other
 *    node N_A + its ordinal among non-author nodes.  Rows < N_A are the
 *    PathSim sources/targets (DPathSim_APVPA.py:18-22).
 *  - node_colid[n]: paper ordinal for paper-typed nodes, mid (venue) ordinal
 *    for mid-typed nodes, -1 otherwise.
 *  - node_type[n]: DPS_T_AUTHOR / DPS_T_PAPER / DPS_T_MID / DPS_T_OTHER.
 *  - edge_rel[e]: DPS_R_AP (relationship 'author_of'), DPS_R_PX ('submit_at'
 *    for APVPA), DPS_R_OTHER.
 */
#ifndef DPATHSIM_H
#define DPATHSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPS_ABI_VERSION 4

enum {
  DPS_OK = 0,
  DPS_ERR_INVALID = -1,    /* bad argument / shape */
  DPS_ERR_HIP = -2,        /* HIP runtime error */
  DPS_ERR_WORKSPACE = -3,  /* workspace too small or misaligned */
  DPS_ERR_OVERFLOW = -4,   /* value does not fit the engine's integer widths */
  DPS_ERR_UNSUPPORTED = -5 /* parameter outside the supported range (e.g. k) */
};

enum { DPS_T_OTHER = 0, DPS_T_AUTHOR = 1, DPS_T_PAPER = 2, DPS_T_MID = 3 };
enum { DPS_R_OTHER = 0, DPS_R_AP = 1, DPS_R_PX = 2 };

/* Stats slots written by dps_global_walks (int64 device array, DPS_STATS_LEN). */
enum {
  DPS_STAT_MAX_C = 0,     /* max C[x,v] over author rows */
  DPS_STAT_MAX_DIAG = 1,  /* max M[x,x] = sum_v C[x,v]^2 over author rows */
  DPS_STAT_MAX_G = 2,     /* max g[x] over author rows */
  DPS_STAT_NNZ_C = 3,     /* nnz of C (author rows) */
  DPS_STATS_LEN = 8
};

int dps_abi_version(void);
const char* dps_last_error(void);

/* Explicit, process-wide tuning overrides for tests and A/B runs (the library
 * reads no environment variables; every value 0 = automatic, the default):
 *   DPS_TUNE_WAVES_PER_ROW  1, 4 or 8 waves share one source row in the hot
 *                           kernel (automatic: 1 for tile_w <= 8192);
 *   DPS_TUNE_TILE_BUILD     1 = block-local, 2 = global-atomic C^T tile build
 *                           (automatic: by the number of mids);
 *   DPS_TUNE_BANK_ORDER     1 = order each C^T bucket's 16-bit entries for the
 *                           hot kernel's LDS banks, 2 = keep the build order
 *                           (automatic: see dps_ct_tiles_build);
 *   DPS_TUNE_LEAN_WPC       1..32 one-wave workgroups per CU in the grid of the
 *                           hot kernel's lean form (automatic: as many as its
 *                           LDS and registers keep resident at once).
 * No reference counterpart (Spark picks its own plans). */
enum { DPS_TUNE_WAVES_PER_ROW = 1, DPS_TUNE_TILE_BUILD = 2, DPS_TUNE_BANK_ORDER = 3,
       DPS_TUNE_LEAN_WPC = 4, DPS_TUNE_KEYS = 5 };
int dps_set_tuning(int32_t key, int32_t value);
int dps_get_tuning(int32_t key);
/* Number of visible HIP devices (hipGetDeviceCount); < 0 on error. */
int dps_device_count(void);

/* ---------------------------------------------------------------------------
 * A2. Typed incidence extraction.
 * Replaces the motif's typed edge filters DPathSim_APVPA.py:78-84 (and
 * :99-105) over the edge/vertex DataFrames of :160-163:
 *   AP pair (node_rowid[src], node_colid[dst]) for every edge with
 *       edge_rel == DPS_R_AP and node_type[dst] == DPS_T_PAPER (src type NOT
 *       checked, as in the reference);
 *   PX pair (node_colid[src], node_colid[dst]) for every edge with
 *       edge_rel == DPS_R_PX, node_type[src] == PAPER, node_type[dst] == MID.
 * Duplicates are kept here (removed by dps_csr_build = the motif's distinct,
 * :86).  Pair order is unspecified.  ap_* / px_* need capacity n_edges.
 * n_ap / n_px: int64 device scalars (written, not accumulated).
 * ------------------------------------------------------------------------- */
int dps_extract_incidence(const int32_t* edge_src, const int32_t* edge_dst,
                          const uint8_t* edge_rel, int64_t n_edges,
                          const uint8_t* node_type, const int32_t* node_rowid,
                          const int32_t* node_colid, int64_t n_nodes,
                          int32_t* ap_row, int32_t* ap_col, int64_t* n_ap,
                          int32_t* px_row, int32_t* px_col, int64_t* n_px,
                          void* stream);

/* ---------------------------------------------------------------------------
 * A2/A3. Typed CSR build = sort + unique (the motif's select('*').distinct(),
 * DPathSim_APVPA.py:86,107, which makes incidences binary -- SURVEY.md K3).
 * Input: n_pairs (row, col) pairs; n_pairs is read from the device scalar
 * `n_pairs_dev` if non-NULL (then `n_pairs` is the capacity), else `n_pairs`.
 * Output: row_ptr int64[n_rows+1], col_out int32[capacity n_pairs] sorted
 * ascending within each row, no duplicates; *nnz_out (int64 device scalar).
 * ------------------------------------------------------------------------- */
size_t dps_csr_build_workspace_size(int64_t n_pairs, int64_t n_rows);
int dps_csr_build(const int32_t* rows, const int32_t* cols, int64_t n_pairs,
                  const int64_t* n_pairs_dev, int64_t n_rows,
                  int64_t* row_ptr, int32_t* col_out, int64_t* nnz_out,
                  void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * A3. Author-venue count matrix C = W_AP . W_PX (the join A->P->V of the motif,
 * DPathSim_APVPA.py:72-74): C[a,v] = |{p : (a,p) in AP, (p,v) in PX}|.
 * Expand-sort-compress SpGEMM, two phases:
 *   symbolic (c_col == NULL): fills c_ptr int64[n_out_rows+1]; *c_nnz = nnz.
 *   numeric  (c_col != NULL): needs c_ptr from the symbolic call; writes
 *            c_col int32[nnz] (ascending per row) and c_val int32[nnz].
 * Output row i is AP row `rows[i]` if `rows` != NULL, else AP row i.
 * `expand_cap` must be >= the expanded size sum_rows sum_{p in AP[row]} |PX[p]|
 * returned by dps_spgemm_expand_size (int64 device scalar; the host reads it
 * to size the workspace).  The numeric call must get the same, unmodified
 * workspace as the preceding symbolic call (it holds the sorted runs).
 * ------------------------------------------------------------------------- */
int dps_spgemm_expand_size(const int64_t* ap_ptr, const int32_t* ap_col, const int32_t* rows,
                           int64_t n_out_rows, const int64_t* px_ptr, int64_t* e_total,
                           void* stream);
size_t dps_spgemm_workspace_size(int64_t n_out_rows, int64_t expand_cap);
int dps_spgemm_count(const int64_t* ap_ptr, const int32_t* ap_col,
                     const int32_t* rows, int64_t n_out_rows,
                     const int64_t* px_ptr, const int32_t* px_col, int64_t n_papers,
                     int64_t* c_ptr, int32_t* c_col, int32_t* c_val, int64_t* c_nnz,
                     int64_t expand_cap, void* ws, size_t ws_bytes, void* stream);

/* A3, the engine's SpGEMM: wavefront-cooperative hash SpGEMM for the same C
 * (output row i = AP row rows[i], or i when rows == NULL; columns ascending).
 * No expanded intermediate array: per row, L = sum_{p in AP[row]} |PX[p]|
 * picks a lane (L <= 16: register sorting network), a workgroup with an LDS
 * hash table (L <= 4096) or a workgroup sorting in a global scratch region
 * (L > 4096).  Two enqueue-only phases with one workspace:
 *   symbolic (c_col == NULL): c_ptr int64[n_out_rows+1], *c_nnz (device);
 *   numeric  (c_col != NULL): c_col/c_val int32[nnz] -- same, unmodified ws.
 * max_row_expand >= max over rows of L (a host bound, e.g. from the raw
 * edges); a row beyond it sets *status_dev = DPS_ERR_OVERFLOW (nullable). */
size_t dps_spgemm_hash_workspace_size(int64_t n_out_rows, int64_t max_row_expand);
int dps_spgemm_hash(const int64_t* ap_ptr, const int32_t* ap_col, const int32_t* rows,
                    int64_t n_out_rows, const int64_t* px_ptr, const int32_t* px_col,
                    int64_t max_row_expand, int64_t* c_ptr, int32_t* c_col, int32_t* c_val,
                    int64_t* c_nnz, int32_t* status_dev, void* ws, size_t ws_bytes, void* stream);

/* A3 when every paper has at most one mid (APVPA: one venue per paper): the
 * expansion of row a IS its AP segment with each paper replaced by its mid,
 * so C comes from one coalesced gather per AP entry plus a segmented sort +
 * unique over the AP rows (a paper -> mid map of n_papers entries first makes
 * that gather one random read).  Output rows = AP rows [0, n_out_rows) (ap_ptr with
 * n_out_rows + 1 entries; the AP CSR must cover exactly these rows).
 * nnz_ap_cap >= ap_ptr[n_out_rows] sizes the workspace.  n_mids: every
 * px_col value is below it (rows longer than 64 are then reduced by an LDS
 * histogram instead of a sort when n_mids <= 8192; 0 = unknown, always sort).
 * Same two phases as dps_spgemm_hash.  A paper with two or more mids is a caller error (the
 * engine chooses this path only when the raw edges give no paper two). */
size_t dps_spgemm_single_workspace_size(int64_t n_out_rows, int64_t nnz_ap_cap,
                                        int64_t n_papers);
int dps_spgemm_single(const int64_t* ap_ptr, const int32_t* ap_col, int64_t n_out_rows,
                      int64_t nnz_ap_cap, const int64_t* px_ptr, const int32_t* px_col,
                      int64_t n_papers, int64_t n_mids, int64_t* c_ptr, int32_t* c_col,
                      int32_t* c_val, int64_t* c_nnz, void* ws, size_t ws_bytes, void* stream);

/* The same with the paper -> mid map given (vp int32 [n_papers], INT_MAX = no
 * mid); px_ptr / px_col are then unused (may be NULL).  Same workspace. */
int dps_spgemm_single_map(const int64_t* ap_ptr, const int32_t* ap_col, int64_t n_out_rows,
                          int64_t nnz_ap_cap, const int32_t* vp, const int64_t* px_ptr,
                          const int32_t* px_col, int64_t n_papers, int64_t n_mids,
                          int64_t* c_ptr, int32_t* c_col, int32_t* c_val, int64_t* c_nnz,
                          void* ws, size_t ws_bytes, void* stream);

/* Paper -> mid map from the typed PX pairs of dps_extract_incidence (capacity
 * n_px_cap, count in the device scalar n_px_dev if non-NULL), without a PX CSR:
 * valid when no paper has two raw PX edges (the single-mid case; the distinct
 * of :86 is then a no-op).  vp int32 [n_papers], INT_MAX where no mid. */
int dps_paper_mid_map(const int32_t* px_paper, const int32_t* px_mid, int64_t n_px_cap,
                      const int64_t* n_px_dev, int64_t n_papers, int32_t* vp, void* stream);

/* ---------------------------------------------------------------------------
 * A4. Global walk ingredients.
 * dps_mid_walks: s[v] = sum over ALL AP rows r of C[r,v]
 *   = sum_{(p,v) in PX} indeg_AP(p)  (author_2 unconstrained in the global
 *   walk motif, DPathSim_APVPA.py:70-84).  s int64[n_mids], fully written.
 * dps_global_walks: g[x] = sum_v C[x,v] * s[v] (metapath_global_walk :70-88),
 *   diag[x] = M[x,x]; stats int64[DPS_STATS_LEN] (see DPS_STAT_*), written.
 * ------------------------------------------------------------------------- */
int dps_mid_walks(const int64_t* ap_ptr, const int32_t* ap_col, int64_t n_ap_rows,
                  const int64_t* px_ptr, const int32_t* px_col, int64_t n_papers,
                  int64_t n_mids, int32_t* paper_indeg_ws, int64_t* s,
                  void* stream);
int dps_global_walks(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                     int64_t n_rows, const int64_t* s, int64_t* g, int64_t* diag,
                     int64_t* stats, void* stream);
/* s from C itself: s[v] = sum_{r < n_rows} C[r,v] (int64[n_mids], written).
 * With C built over EVERY AP row (authors and untyped author_of sources) this
 * equals dps_mid_walks' s without the per-paper in-degree pass; the engine
 * builds C that way. */
int dps_col_sums(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                 int64_t n_rows, int64_t n_mids, int64_t* s, void* stream);

/* Work estimate per source row of the hot kernel (used to order rows heaviest
 * first and to balance row shards across ranks):
 * terms[x] = sum_{v : C[x,v] > 0} n_v with n_v = nnz of column v over rows
 * [0, n_rows) -- the C^T entries row x's scatter reads.  col_count_ws:
 * uint32[n_mids] scratch (left holding n_v).  No reference counterpart (the
 * reference has no work partitioning). */
int dps_row_work(const int64_t* c_ptr, const int32_t* c_col, int64_t n_rows, int64_t n_mids,
                 uint32_t* col_count_ws, int64_t* terms, void* stream);

/* A4 fused (what the engine runs every build): s = column sums of C over rows
 * [0, n_rows) (dps_col_sums), n_v = entries per mid over the author rows
 * [0, n_authors) (uint32 [n_mids]), then over the author rows g, diag
 * (nullable), the row work terms[x] = sum_{v in x} n_v (nullable; as
 * dps_row_work) and stats (nullable) -- two passes over C instead of four. */
int dps_walks_fused(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                    int64_t n_rows, int64_t n_authors, int64_t n_mids, int64_t* s,
                    uint32_t* n_v, int64_t* g, int64_t* diag, int64_t* terms, int64_t* stats,
                    void* stream);
/* The same with a workspace (dps_walks_workspace_size(nnz_cap, n_mids) bytes,
 * 256-byte aligned; nnz_cap >= nnz C, e.g. the SpGEMM output capacity): with
 * more mids than one LDS range the column sums bucket C's entries by mid range
 * once instead of re-reading C per range.  ws == NULL: as dps_walks_fused.
 * Memory: the bucketed path holds one 8-byte pair per C entry (8 B x nnz_cap)
 * plus per-range counts; with at most 6144 mids, or more than 4096 x 12288,
 * the workspace is 256 bytes and the call takes the unbucketed path. */
size_t dps_walks_workspace_size(int64_t nnz_cap, int64_t n_mids);
int dps_walks_fused_ws(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                       int64_t n_rows, int64_t n_authors, int64_t n_mids, int64_t* s,
                       uint32_t* n_v, int64_t* g, int64_t* diag, int64_t* terms, int64_t* stats,
                       int64_t nnz_cap, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * A5 operand layout, step 1: target relabeling (a pure layout choice; results
 * never depend on it).  Targets are relabeled in ascending global walk g (ties
 * by original index) with a stable LSD radix sort over the low key_bits bits
 * of g (key_bits >= bit length of max g).  Outputs: t_perm[label] = original,
 * t_rank[original] = label, g_t[label] = g[t_perm[label]] (all n_targets).
 * ------------------------------------------------------------------------- */
size_t dps_target_order_workspace_size(int64_t n_targets);
int dps_target_order(const int64_t* g, int64_t n_targets, int32_t key_bits,
                     int32_t* t_perm, int32_t* t_rank, int64_t* g_t,
                     void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * A5 operand layout, step 2: target-tiled transpose of C for the C.C^T kernels.
 * Target labels (t_rank[y], or y if t_rank == NULL) in [0, n_targets) are cut
 * into tiles of `tile_w` (a power of two, 256..65536, or the T15 widths 7680 /
 * 15360; the hot kernel keeps one tile's packed counters in LDS: u8 at tile_w
 * 8192 / 7680, 4-bit at 16384 / 15360 -- the T15 widths take 7680 bytes, so 20
 * one-wave workgroups stay resident per CU instead of 18).  Bucket
 * (v, t) holds, for every y of tile t with C[y,v] > 0, packed entries in one of
 * three formats, l = label(y) - t*tile_w:
 *   tile_w <= 8192 (and 7680):  uint16 (l << 3) | e, one piece of value 2^e: C[y,v] is
 *                    split into power-of-two pieces that sum to it (as many
 *                    2^emax as fit, then the set bits of the rest), emax = 7,
 *                    or 5 when l % 4 == 3 (e = 6, 7 at l % 4 == 3 are padding
 *                    codes).  The low five bits 8*(l % 4) + e are the shift
 *                    that adds C[x,v]*2^e to target l's byte of a packed-u8
 *                    dword;
 *   tile_w 16384 / 15360: uint16 (l << 2) | e, the same for packed 4-bit counters:
 *                    emax = 3, or 1 when l % 8 == 7 (e = 2, 3 at l % 8 == 7 are
 *                    padding codes); low five bits 4*(l % 8) + e;
 *   tile_w >= 32768: uint32 (C[y,v] << 16) | l, one entry per (y, v).
 * To decode a 16-bit entry h: l = h >> 3 (resp. >> 2), value = 1 << (h & 7)
 * (resp. & 3), skipping padding codes; summing the values of one (v, l) gives
 * C[y,v].  16-bit entries are packed two per uint32 word, the first in the low
 * half.  Buckets are stored contiguously in [v][t] order: bucket (v,t) is the
 * uint32 words tile_ent[tile_off[v*T + t] .. tile_off[v*T + t + 1]),
 * T = ceil(n_targets/tile_w).  Every bucket is padded to 16 bytes (32-bit:
 * C = 0 entries; 16-bit: groups of padding codes on one dword -- {7,7} / {7,6,6}
 * at u8, {3,3} / {3,2,2} at 4-bit, each group at one label of a dword's last
 * target (l % 4 == 3, resp. l % 8 == 7) -- which add
 * C * 2^32 == 0 to the packed accumulators), so bucket starts are 16-byte
 * aligned and 16-byte chunks never straddle buckets.  tile_off
 * uint32[n_mids*T + 1] (word offsets), tile_ent uint32[dps_ct_tiles_ent_capacity()].
 * Optional: tile_maxc uint32[n_mids*T + 1] = max C[y,v] per bucket;
 * tile_gmin int64[T] = min g[y] per tile (needs g).
 * Requires max C <= 65535 (else *status_dev = DPS_ERR_OVERFLOW).  Entry order
 * inside a bucket is unspecified (results are exact integer sums).
 * ------------------------------------------------------------------------- */
size_t dps_ct_tiles_workspace_size(int64_t n_mids, int64_t n_targets, int32_t tile_w);
/* The same build with a host bound nnz_cap >= nnz(C[0:n_targets]) (e.g. the
 * raw-edge expansion count): with many mids (more than 8 * 8192) the buckets
 * are laid out from ONE stable radix sort of (bucket, entry) pairs instead of
 * per-entry global atomics on n_mids*T bucket counters (config4, 200 k
 * topics); otherwise identical to dps_ct_tiles_build.  Same outputs and
 * format; ws from dps_ct_tiles_workspace_size2.  A bound below the real nnz is
 * detected on the device: *status_dev = DPS_ERR_OVERFLOW, the outputs are then
 * undefined and nothing is written past the workspace. */
size_t dps_ct_tiles_workspace_size2(int64_t n_mids, int64_t n_targets, int32_t tile_w,
                                    int64_t nnz_cap);
int dps_ct_tiles_build2(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                        const int64_t* g, const int32_t* t_rank, int64_t n_targets, int64_t n_mids,
                        int32_t tile_w, int64_t nnz_cap, uint32_t* tile_off, uint32_t* tile_ent,
                        uint32_t* tile_maxc, int64_t* tile_gmin, int32_t* status_dev, void* ws,
                        size_t ws_bytes, void* stream);
/* Both tile sets the bench shape's hot kernel reads, from one walk of C (round
 * 6): the 4-bit tiles at tile_w (16384 or 15360: tile_off / tile_ent /
 * tile_maxc / tile_gmin) and their companion u8 tiles at tile_w / 2 (half_off /
 * half_ent / half_maxc, no minima) -- bit for bit the outputs of two
 * dps_ct_tiles_build2 calls (offsets and maxima; entries as multisets per
 * bucket), which it makes itself with many mids (more than 8 * 8192) or when
 * the entry buffers' sizes (tile_ent_words / half_ent_words, uint32 words) reach
 * 2^31.  Overflow (max C > 65535) goes to *status_dev; *half_status is zeroed
 * (and set only by the two-call path).  hv_c (optional, with hv_slot / n_hv
 * from dps_heavy_venues): the venue-skipping table of dps_heavy_table, written
 * by the same walk (zeroed with the build's counters) when n_hv is even and
 * hv_c 4-byte aligned, else by a dps_heavy_table call.  ws:
 * dps_ct_tiles_workspace_size_dual (0 for other widths).  Replaces nothing in
 * the reference (layout only); A5's operand build, DPathSim_APVPA.py:90-109. */
size_t dps_ct_tiles_workspace_size_dual(int64_t n_mids, int64_t n_targets, int32_t tile_w,
                                        int64_t nnz_cap);
int dps_ct_tiles_build_dual(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                            const int64_t* g, const int32_t* t_rank, int64_t n_targets,
                            int64_t n_mids, int32_t tile_w, int64_t nnz_cap, uint32_t* tile_off,
                            uint32_t* tile_ent, int64_t tile_ent_words, uint32_t* tile_maxc,
                            int64_t* tile_gmin, uint32_t* half_off, uint32_t* half_ent,
                            int64_t half_ent_words, uint32_t* half_maxc, int32_t* status_dev,
                            int32_t* half_status, const int32_t* hv_slot, int32_t n_hv,
                            uint16_t* hv_c, void* ws, size_t ws_bytes, void* stream);
/* Per-bucket count sums of built tiles: tile_sum[b] = sum over the bucket's
 * entries of their values (2^e of a 16-bit piece, padding codes excluded; C of
 * a 32-bit entry) = sum_{y of tile t} C[y,v] for bucket b = v*T + t, b <
 * n_buckets = n_mids*T.  uint32 [n_buckets]. */
int dps_ct_tiles_sums(const uint32_t* tile_off, const uint32_t* tile_ent, int64_t n_buckets,
                      int32_t tile_w, uint32_t* tile_sum, void* stream);
/* uint32 words tile_ent must hold for nnz = nnz(C[0:n_targets]) and any
 * sum_c >= the sum of those entries' values (e.g. sum(s)): padding included,
 * plus one spare 16-byte chunk.  0 if sum_c < nnz. */
int64_t dps_ct_tiles_ent_capacity(int64_t nnz, int64_t sum_c, int64_t n_mids,
                                  int64_t n_targets, int32_t tile_w);
int dps_ct_tiles_build(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                       const int64_t* g, const int32_t* t_rank,
                       int64_t n_targets, int64_t n_mids, int32_t tile_w,
                       uint32_t* tile_off, uint32_t* tile_ent, uint32_t* tile_maxc,
                       int64_t* tile_gmin, int32_t* status_dev,
                       void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Hot-kernel extensions, passed as one host struct (dps_cct_ext, nullable):
 *
 * (1) Companion u8 tiles for tile_w = 16384.  The 16384-target tiles carry
 *   16-bit entries for packed 4-bit counters (dps_ct_tiles_build); a tile
 *   whose per-row bound exceeds 15 needs wider counters.  With half_off /
 *   half_ent / half_maxc = dps_ct_tiles_build of the SAME C and t_rank at
 *   tile_w 8192, such a tile runs as its two 8192-target halves from those u8
 *   tiles; without them it takes wide 4-bit passes (slower, same results).
 *
 * (2) Venue skipping (an exact pruning; no reference
 * counterpart -- the reference counts every path of the motif,
 * DPathSim_APVPA.py:90-109).  With the row-sum denominator every target has
 * g[y] = sum_v C[y,v] s[v] (metapath_global_walk :70-88), so once a
 * row's top-k is full (k-th score tau) the heavy venues h with
 * 2 C[x,h] <= tau s[h] cannot lift a target to tau on their own: the kernel
 * stops scattering their buckets, flags targets from the other venues' counts
 * with a threshold lowered by max_h C[x,h]/s[h] * g[y], and completes each
 * flagged target's count exactly from a dense table of C over the heavy venues
 * before scoring it.  Results are identical with and without it.
 *
 * dps_heavy_venues: hv_slot int32[n_mids] = slot in [0, n_hv) of up to n_hv
 *   venues with the most author entries n_v (dps_walks_fused's n_v), -1 for
 *   every other venue (and for n_v == 0).  1 <= n_hv <= 64.
 * dps_heavy_table: hv_c uint16[n_targets * n_hv] (written whole): entry
 *   label(y) * n_hv + hv_slot[v] = C[y,v] for every author row y < n_targets
 *   and heavy venue v, 0 elsewhere; label(y) = t_rank[y] (NULL = y).  Needs
 *   max C <= 65535 (the engine's check).
 * Venue skipping is valid ONLY when the top-k call's g is the row-sum global
 *   walk g = C.s for this s (not with the diag denominator); hv_c must use the
 *   same t_rank.  Used by the one-wave kernel (tile_w 8192 and 16384); other
 *   tile widths ignore it.
 * ------------------------------------------------------------------------- */
typedef struct dps_cct_ext {
  /* (2) venue skipping; s == NULL: off */
  const int64_t* s;          /* s[v] = column sums of C over every AP row (dps_walks_fused) */
  const int32_t* hv_slot;    /* [n_mids], dps_heavy_venues */
  const uint16_t* hv_c;      /* [n_targets * n_hv], dps_heavy_table */
  int32_t n_hv;              /* 1..64 */
  /* (1) companion u8 tiles (tile_w 16384 only); half_ent == NULL: off */
  const uint32_t* half_off;
  const uint32_t* half_ent;
  const uint32_t* half_maxc;
  /* (3) optimistic 4-bit passes (with (1) only; NULL: off): tile_sum = the
   * per-bucket count sums of the COMPANION u8 tiles (dps_ct_tiles_sums over
   * half_off / half_ent at 8192).  A 16384-target tile whose bound exceeds 15
   * (up to 255) then takes ONE 4-bit pass; a count that reached 16 is detected
   * exactly, per 8192-target half, from the digit sum of that half's counters,
   * and only such a half runs again as its u8 half tile.  Same results, fewer
   * accumulator passes. */
  const uint32_t* tile_sum;
} dps_cct_ext;
int dps_heavy_venues(const uint32_t* n_v, int64_t n_mids, int32_t n_hv, int32_t* hv_slot,
                     void* stream);
int dps_heavy_table(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                    const int32_t* t_rank, int64_t n_targets, const int32_t* hv_slot, int32_t n_hv,
                    uint16_t* hv_c, void* stream);

/* ---------------------------------------------------------------------------
 * ★ A5+A6+A7 fused: the hot kernel.  For every source row x in
 * [row_begin, row_end) (original author ordinals): M[x,y] = C[x,:].C[y,:] over
 * all targets y != x (metapath_pairwise_walk :90-109), score =
 * (double)(2*M) / (double)(g[x]+g[y]) (one IEEE division, :51-52; 0/0 -> 0.0),
 * and the top-k targets by (score desc, original y asc), self excluded
 * (:18-22).  Slots beyond the n_targets-1 available targets: idx -1, cnt 0,
 * score 0.0.  g: original order; g_t/t_perm/t_rank: the relabeling of
 * dps_target_order (all NULL = identity labels, g_t = g); tile_* from
 * dps_ct_tiles_build with the same t_rank (tile_gmin required, tile_maxc
 * optional -- enables skipping tiles that cannot hold a top-k candidate);
 * ext: companion u8 tiles / venue skipping (above), NULL = neither.
 * Outputs (row-major [row_end-row_begin][k], output row x - row_begin):
 * out_idx int32 (original ordinals), out_cnt int64 (M), out_score double.
 * 1 <= k <= 256.  row_order (nullable, int32[row_end-row_begin]): a
 * permutation of [row_begin, row_end) giving the order in which rows are
 * dequeued (heaviest first keeps the kernel tail short); results never
 * depend on it.
 * Requires max M[x,x] < 2^31.  ws: dps_cct_topk_workspace_size() bytes.
 * ------------------------------------------------------------------------- */
size_t dps_cct_topk_workspace_size(void);
int dps_cct_topk(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                 const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                 const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                 const uint32_t* tile_off, const uint32_t* tile_ent,
                 const uint32_t* tile_maxc, const int64_t* tile_gmin, const dps_cct_ext* ext,
                 int64_t row_begin, int64_t row_end, const int32_t* row_order, int32_t k,
                 int32_t* out_idx, int64_t* out_cnt, double* out_score,
                 void* ws, size_t ws_bytes, void* stream);

/* The same for an arbitrary list of source rows (any order, repeats allowed):
 * output row i is rows[i] (rows[i] in [0, n_targets)), and rows are dequeued
 * in list order, so a caller passes them heaviest first.  Used for row-sampled
 * parity runs and for non-contiguous shards. */
int dps_cct_topk_rows(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                      const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                      const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                      const uint32_t* tile_off, const uint32_t* tile_ent,
                      const uint32_t* tile_maxc, const int64_t* tile_gmin,
                      const dps_cct_ext* ext, const int32_t* rows,
                      int64_t n_rows, int32_t k, int32_t* out_idx, int64_t* out_cnt,
                      double* out_score, void* ws, size_t ws_bytes, void* stream);

/* Load balance for the hot kernel (one wave owns one row, so a single very
 * heavy row would bound a launch's time -- the N-GPU shards in particular):
 *
 * dps_cct_topk_split: one launch over [row_begin, row_end) whose dequeue list
 *   row_order[0 .. n_order) starts with n_pieces row PIECES -- slot i <
 *   n_pieces is source row row_order[i] restricted to the target tiles
 *   [piece_t0[i], piece_t1[i]) (tile = tile_w consecutive target labels, T =
 *   ceil(n_targets/tile_w)); its ranked targets (score > 0, order score desc
 *   then y asc, -1 after them, no zero-score fill) go to row i of piece_* --
 *   followed by whole rows, written to output row x - row_begin of out_* as
 *   dps_cct_topk writes them.  Rows of the range listed neither way are left
 *   untouched.  The pieces of one row must cover [0, T) exactly once.
 * dps_topk_merge: for every group m of pieces_per_row consecutive piece slots
 *   (all of one row x = rows[m * pieces_per_row]), merges their lists into the
 *   row's exact top-k (the top-k of a union is the top-k of the members'
 *   top-ks), adds the zero-score fill in reference order and -1, and writes
 *   output row x - row_begin of out_*.  1 <= pieces_per_row <= 64. */
int dps_cct_topk_split(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                       const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                       const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                       const uint32_t* tile_off, const uint32_t* tile_ent,
                       const uint32_t* tile_maxc, const int64_t* tile_gmin,
                       const dps_cct_ext* ext, int64_t row_begin,
                       int64_t row_end, const int32_t* row_order, int64_t n_order,
                       const int32_t* piece_t0, const int32_t* piece_t1, int64_t n_pieces,
                       int32_t* piece_idx, int64_t* piece_cnt, double* piece_score, int32_t k,
                       int32_t* out_idx, int64_t* out_cnt, double* out_score, void* ws,
                       size_t ws_bytes, void* stream);
int dps_topk_merge(const int32_t* piece_idx, const int64_t* piece_cnt, const double* piece_score,
                   const int32_t* rows, int64_t n_groups, int32_t pieces_per_row, int32_t k,
                   int64_t n_targets, int64_t row_begin, int32_t* out_idx, int64_t* out_cnt,
                   double* out_score, void* stream);

/* ★ Symmetric all-pairs top-k: the same lists as dps_cct_topk over every row
 * [0, n_targets), with each pair (x, y) scanned once instead of twice (M[x,y] =
 * M[y,x], the score's denominator is symmetric too).  Targets are labelled by
 * ascending g and cut into tiles of tile_w (8192 or 16384; one-wave kernel, no
 * venue skipping).  Row x in tile a:
 *   1. band pass: x over the tiles [a - band, a + band] (heavy-first order
 *      row_order, may be NULL), its band list into out_*;
 *   2. rest pass, rows in descending label order: rows whose band list holds
 *      k positive scores ("strong") continue over the tiles above a + band
 *      with the band's k-th score as the threshold; the others scan every tile.  A pair with y in a tile above a + band is
 *      seen by x alone: it becomes a record (y <- x, M) when its score reaches
 *      y's band k-th score (rounded down to fp32), which bounds y's final k-th
 *      score from below, so no pair of y's top-k is lost;
 *   3. each strong row's band list, rest-pass list and records merge into its
 *      exact top-k (order score desc, then target ordinal asc).
 * rec_cap bounds the records (workspace: dps_cct_sym_workspace_size); the
 * number emitted is written to *rec_stat (device) -- above rec_cap the lists
 * are incomplete and the call must be repeated with a larger rec_cap.  ws is
 * dps_cct_topk's counter workspace (words 1-3: both passes' counts).
 * Replaces the same reference loop as dps_cct_topk (DPathSim_APVPA.py:36,
 * 90-109, 51-52). */
size_t dps_cct_sym_workspace_size(int64_t n_targets, int32_t k, int64_t rec_cap);
int dps_cct_sym(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                const int64_t* g, const int64_t* g_t, const int32_t* t_perm,
                const int32_t* t_rank, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                const uint32_t* tile_off, const uint32_t* tile_ent, const uint32_t* tile_maxc,
                const int64_t* tile_gmin, const dps_cct_ext* ext, const int32_t* row_order,
                int32_t band, int64_t rec_cap, int32_t k, int32_t* out_idx, int64_t* out_cnt,
                double* out_score, unsigned long long* rec_stat, void* sym_ws, size_t sym_ws_bytes,
                void* ws, size_t ws_bytes, void* stream);

/* Heavy-first dequeue list for dps_cct_topk / dps_cct_topk_split (no
 * counterpart in the reference; load balance of the all-pairs loop :36):
 * rows row_begin + [0, n_rows) ordered by work[i] descending on a log scale
 * (four steps per octave, equal steps in row order), the first n_split of them
 * repeated `pieces` times in front -- dq has n_rows + n_split * (pieces - 1)
 * entries.  Any order gives identical top-k results. */
size_t dps_heavy_first_workspace_size(int64_t n_rows);
int dps_heavy_first(const int64_t* work, int64_t n_rows, int64_t row_begin, int64_t n_split,
                    int32_t pieces, int32_t* dq, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Single-source row (the reference's run() loop, :30-50): for one sparse C row
 * (src_col/src_val, src_len entries, device), the dense pairwise walk
 * out_m[y] = sum_v C[src,v] * C[y,v] for all targets y, in ORIGINAL target
 * order (int64[n_targets]); t_perm as for dps_cct_topk (NULL = identity).
 * ------------------------------------------------------------------------- */
int dps_walk_row(const int32_t* src_col, const int32_t* src_val, int64_t src_len,
                 const int32_t* t_perm, int64_t n_targets, int64_t n_mids, int32_t tile_w,
                 const uint32_t* tile_off, const uint32_t* tile_ent,
                 int64_t* out_m, void* stream);

/* The reference's per-target score (:51-52) for one source row on the device:
 * score[y] = (double)(2*m[y]) / (double)(gx + g[y]) (one IEEE division);
 * *zero_div (int64 device scalar, may be NULL) counts targets with
 * gx + g[y] == 0, where the reference raises ZeroDivisionError (score 0.0). */
int dps_row_scores(const int64_t* m, const int64_t* g, int64_t gx, int64_t n, double* score,
                   int64_t* zero_div, void* stream);

/* metapath_pairwise_walk(source, target) (:90-109) for two sparse C rows with
 * ascending columns: *out = sum_v a[v]*b[v] (int64 device scalar). */
int dps_pair_count(const int32_t* a_col, const int32_t* a_val, int64_t a_len,
                   const int32_t* b_col, const int32_t* b_val, int64_t b_len,
                   int64_t* out, void* stream);

/* ---------------------------------------------------------------------------
 * Row sharding across ranks (no counterpart in the reference,
 * whose Spark session :146-168 brings each .count() of :86/:107 back to the
 * driver).  Device arrays, enqueued on `stream`, nothing read back:
 * dps_shard_edges: contiguous shards of (nearly) equal work for `world` ranks:
 *   work[i] = terms[i] + (sum(terms) / n_rows) / 2 (terms = the build's row
 *   work, dps_walks_fused), edges[r] (int64 [world + 1]) = the number of rows
 *   whose inclusive work prefix is <= r * total / world (edges[0] = 0,
 *   edges[world] = n_rows).  With edges_ref, *mismatch += the number of r with
 *   edges[r] != edges_ref[r] (a plan check inside a timed step).  1 <= world
 *   <= 255; ws from dps_shard_edges_workspace_size(n_rows).
 * dps_pack_counts: out[i] = (cnt[i] << 32) | (uint32)idx[i], the 8-byte wire
 *   word of one top-k slot (the root rebuilds the score).
 * dps_unpack_gathered: rows x in [edges[0], edges[world]) of the gathered
 *   [world * m, k] words (rank r's rows at r * m), x at gathered row r * m +
 *   x - edges[r]: out_idx / out_cnt [n_rows, k] and out_score = double(2 cnt) /
 *   double(den[x] + den[idx]) -- the hot kernel's division of the same exact
 *   integers (:51-52), bit-identical -- 0.0 for empty (-1) or zero-count slots.
 *   n_rows must equal edges[world] - edges[0]; the kernel never writes past
 *   n_rows rows nor reads past a shard's m gathered rows if the device edges
 *   disagree (those slots are then left unwritten).
 * ------------------------------------------------------------------------- */
size_t dps_shard_edges_workspace_size(int64_t n_rows);
int dps_shard_edges(const int64_t* terms, int64_t n_rows, int32_t world, int64_t* edges,
                    const int64_t* edges_ref, int64_t* mismatch, void* ws, size_t ws_bytes,
                    void* stream);
int dps_pack_counts(const int32_t* idx, const int64_t* cnt, int64_t n, int64_t* out, void* stream);
int dps_unpack_gathered(const int64_t* gathered, int32_t world, int64_t m, int32_t k,
                        const int64_t* edges, int64_t n_rows, const int64_t* den, int32_t* out_idx,
                        int64_t* out_cnt, double* out_score, void* stream);

/* ---------------------------------------------------------------------------
 * A5 operand layout split across ranks (N > 1).  Each rank
 * builds the C^T tiles of its own target-tile range and the ranks all-gather
 * the slices; C, s, g and the target order stay replicated.  Replaces the
 * per-executor re-join of the whole graph the Spark job does for every target
 * (DPathSim_APVPA.py:72-76 inside the session of :146-168).
 * dps_label_rows: sub-C of the target labels [l0, l1) in label order --
 *   sub_ptr int64[l1-l0+1], row i = C row t_perm[l0+i] (t_perm NULL =
 *   identity) -- so that dps_ct_tiles_build(2) over it with t_rank = NULL,
 *   g = g_t + l0 and n_targets = l1-l0 builds exactly tiles l0/W .. of the
 *   full build (l0 a multiple of tile_w).  sub_col / sub_val capacity: the
 *   rows' total length (e.g. nnz(C)).  ws: dps_label_rows_workspace_size(l1-l0).
 * dps_tiles_slice_words: uint32 words of one rank's slice for n_mids mids,
 *   tiles_per_rank tiles and at most ent_cap entry words.
 * dps_tiles_pack: one rank's build of n_tiles <= tiles_per_rank tiles
 *   (tile_off / tile_maxc [n_mids*n_tiles+1], tile_gmin [n_tiles], tile_ent;
 *   maxc / gmin nullable) into its slice; entries beyond ent_cap words set
 *   *overflow = DPS_ERR_OVERFLOW (nullable) and are not copied.
 * dps_tiles_assemble: the gathered slices (rank r at r * slice_words, rank r
 *   owning tiles [r*tiles_per_rank, ...) of n_tiles) -> the full tile_off /
 *   tile_ent / tile_maxc / tile_gmin of dps_ct_tiles_build, bucket for bucket
 *   (each bucket's entries in the slice build's order); tile_ent holds
 *   ent_words words.  A slice whose offsets leave its capacity, a layout
 *   larger than ent_words, or a nonzero *status on entry (the slice build's
 *   own status) leaves every bucket empty with *status = DPS_ERR_OVERFLOW (or
 *   the status it had): the tiles are never read out of bounds.  ws:
 *   dps_tiles_assemble_workspace_size(n_mids, world).
 * ------------------------------------------------------------------------- */
size_t dps_label_rows_workspace_size(int64_t n);
int dps_label_rows(const int64_t* c_ptr, const int32_t* c_col, const int32_t* c_val,
                   const int32_t* t_perm, int64_t l0, int64_t l1, int64_t* sub_ptr,
                   int32_t* sub_col, int32_t* sub_val, void* ws, size_t ws_bytes, void* stream);
int64_t dps_tiles_slice_words(int64_t n_mids, int64_t tiles_per_rank, int64_t ent_cap);
int dps_tiles_pack(const uint32_t* tile_off, const uint32_t* tile_maxc, const int64_t* tile_gmin,
                   const uint32_t* tile_ent, int64_t n_mids, int64_t n_tiles,
                   int64_t tiles_per_rank, int64_t ent_cap, uint32_t* slice, int32_t* overflow,
                   void* stream);
size_t dps_tiles_assemble_workspace_size(int64_t n_mids, int32_t world);
int dps_tiles_assemble(const uint32_t* gathered, int32_t world, int64_t n_mids, int64_t n_tiles,
                       int64_t tiles_per_rank, int64_t ent_cap, uint32_t* tile_off,
                       uint32_t* tile_ent, int64_t ent_words, uint32_t* tile_maxc,
                       int64_t* tile_gmin, int32_t* status, void* ws, size_t ws_bytes,
                       void* stream);

/* ---------------------------------------------------------------------------
 * RCCL over xGMI: one rank per process and GPU.  Replaces
 * the Spark shuffle that brings results back to the driver (the .count()
 * actions DPathSim_APVPA.py:86,107 over the session of :146-168).
 * dps_comm_get_id: an ncclUniqueId (dps_comm_id_bytes() bytes) on ONE rank;
 *   the caller shares the bytes with the other ranks out of band.
 * dps_comm_init: ncclCommInitRank on the CURRENT device (hipSetDevice first);
 *   *comm_out is opaque.  dps_comm_destroy releases it (NULL is a no-op).
 * dps_bcast: `bytes` bytes of buf from `root` to every rank (in place).
 * dps_gather: every rank's `bytes` bytes of send into recv on `root`, rank r
 *   at recv + r * bytes (recv unused elsewhere).  Device buffers, enqueued on
 *   the caller's stream like every other entry point.
 * ------------------------------------------------------------------------- */
int dps_comm_id_bytes(void);
int dps_comm_get_id(uint8_t* id_out);
int dps_comm_init(void** comm_out, int32_t nranks, int32_t rank, const uint8_t* id);
int dps_comm_destroy(void* comm);
int dps_bcast(void* comm, void* buf, size_t bytes, int32_t root, void* stream);
int dps_gather(void* comm, const void* send, void* recv, size_t bytes, int32_t root, void* stream);
/* dps_allgather: every rank's `bytes` bytes of send into recv on EVERY rank,
 *   rank r at recv + r * bytes (the tile slices of the N > 1 build). */
int dps_allgather(void* comm, const void* send, void* recv, size_t bytes, void* stream);

/* ---------------------------------------------------------------------------
 * A8. Run-log format (DPathSim_APVPA.py:32-67), host-side, for all-pairs
 * results.  Host arrays only (no device work, no GPU needed).
 *
 * dps_format_float: Python's repr() of a double (the reference formats scores
 *   with '{}'.format(float), :47-49/:56-64) into out[cap] (NUL-terminated).
 * dps_write_topk_log: for source rows x = row_begin + r, r < n_rows, writes
 *   "Source author global walk: {g[x]}" and, for each ranked target y =
 *   idx[r*k + s] >= 0 in rank order, the reference's five-line target block
 *   ("Pairwise authors walk {id[y]}: {cnt}", "Target author global walk:
 *   {g[y]}", "Sim score {label[x]} - {label[y]}: {score}", "***Stage done in:
 *   {stage_seconds}", "---"); then "***Overall done in: {overall_seconds}" if
 *   overall_seconds >= 0.  ids / labels: UTF-8 strings of every author ordinal,
 *   concatenated in *_blob with offsets *_off[n_authors + 1].  g_host is indexed
 *   by author ordinal.  append != 0 appends (the reference opens with 'a').
 *   n_threads <= 0: all hardware threads.
 * ------------------------------------------------------------------------- */
int dps_format_float(double v, char* out, size_t cap);
int dps_write_topk_log(const char* path, int append, int64_t row_begin, int64_t n_rows, int32_t k,
                       const int32_t* idx_host, const int64_t* cnt_host, const double* score_host,
                       const int64_t* g_host, const char* id_blob, const int64_t* id_off,
                       const char* label_blob, const int64_t* label_off, double stage_seconds,
                       double overall_seconds, int n_threads);

/* ---------------------------------------------------------------------------
 * f1. Native GEXF scan for read_dblp_nx_file (DPathSim_APVPA.py:114-129, the
 * networkx.read_gexf of :116), host-only.  dps_gexf_open mmaps and scans the
 * file; *status 0 = parsed, 1 = outside the supported subset (nested <nodes>,
 * DOCTYPE, numeric attribute types, undefined attvalue keys, edge-type
 * conflicts, I/O errors): the caller runs its own parser, which reports the
 * reference's exceptions.  dps_gexf_info: 0 nodes, 1 edges, 2 type names,
 * 3 relationship names, 4 directed, 5-8 bytes of node ids / labels / type
 * names / relationship names, 9 bytes of the edge-id buffer.  dps_gexf_export
 * fills caller arrays: string tables as concatenated UTF-8 + int64 offsets
 * [n+1]; lab_null[i] = 1 when the node has no label; ntype / e_rel = -1 when
 * absent (node without node_type, edge without relationship); e_key_off[j] =
 * offset of edge j's NUL-terminated id in key_buf, -1 when it has none.
 * ------------------------------------------------------------------------- */
void* dps_gexf_open(const char* path, int32_t* status);
int64_t dps_gexf_info(void* h, int32_t what);
int dps_gexf_export(void* h, int64_t* id_off, char* id_buf, int64_t* lab_off, char* lab_buf,
                    uint8_t* lab_null, int32_t* ntype, int64_t* type_off, char* type_buf,
                    int32_t* e_src, int32_t* e_dst, int32_t* e_rel, int64_t* e_key_off,
                    char* key_buf, int64_t* rel_off, char* rel_buf);
void dps_gexf_close(void* h);

#ifdef __cplusplus
}
#endif
#endif /* DPATHSIM_H */
