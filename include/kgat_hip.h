/*
 * kgat_hip.h -- C-ABI of the MI355X (gfx950) KGAT / NFM hot-path library
 * (libkgat_hip.so).
 *
 * Every entry point takes plain device pointers + sizes and the caller's
 * hipStream_t (as void*), is stream-ordered and asynchronous, never allocates
 * or frees caller memory, never synchronises the device, and returns an int
 * status: 0 on success, a hipError_t value on a HIP failure, or one of the
 * KGAT_ERR_* codes below.  kgat_strerror() turns a status into text.  No C++
 * exception crosses this boundary.  Scratch memory is caller-provided.
 *
 * The reference has no FFI: its drop-in boundary is the Python module API of
 * src/model/KGAT/model.py and src/model/NFM/model.py.  Each entry below names
 * the reference operation it replaces (paths relative to the reference root);
 * the Python host package binds them with ctypes.
 *
 * Layouts: row-major fp32 tables with a leading dimension (ld, in elements,
 * a multiple of 4, 16-byte aligned base); CSR graphs with int64 row pointers
 * and int32 column ids.
 */
#ifndef KGAT_HIP_H
#define KGAT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  KGAT_OK = 0,
  KGAT_ERR_INVALID = 1001,         /* bad argument (null pointer, negative size, misaligned) */
  KGAT_ERR_UNSUPPORTED_DIM = 1002, /* feature width not in the compiled set */
  KGAT_ERR_WORKSPACE = 1003,       /* caller workspace too small */
  KGAT_ERR_COMM_UNAVAILABLE = 1004, /* no loadable RCCL (kgat_comm_*) */
  KGAT_ERR_COMM_BASE = 1100         /* + ncclResult_t: an RCCL call failed (kgat_comm_*) */
};

/* A CSR matrix plus its load-balancing plan.  Rows whose degree exceeds
 * long_threshold are "long": they are cut into segments of at most seg_len
 * edges (seg_row/seg_beg, grouped per long row by long_seg_off) that are
 * reduced in a deterministic second pass.  Built once per graph structure by
 * kgat_csr_plan() on the host. */
typedef struct kgat_csr {
  const int64_t *rowptr;       /* [n_rows + 1] */
  const int32_t *col;          /* [nnz] */
  const float *val;            /* [nnz] */
  int64_t n_rows;
  int64_t nnz;
  const int32_t *long_rows;    /* [n_long] */
  const int32_t *long_seg_off; /* [n_long + 1], offsets into the segment arrays */
  const int32_t *seg_row;      /* [n_seg] */
  const int64_t *seg_beg;      /* [n_seg] */
  int32_t n_long;
  int32_t n_seg;
  /* the segment length of a fixed-length plan (kgat_csr_plan: every segment but a
   * row's last holds exactly seg_len entries); 0 for a plan whose segments vary in
   * length (kgat_csr_plan_cols).  The SpMM kernels take a segment's end from the
   * next segment's start and accept either; the row softmax's hub-segment
   * arithmetic needs the fixed 512-entry plan and rejects any other. */
  int32_t seg_len;
  int32_t long_threshold;
  /* [4 * ceil(n_seg / 4)] or null (= identity): the segment each launch slot of the
   * SpMM's long-row blocks takes (slot = 4 * block + wave; values >= n_seg are
   * padding).  A scheduling choice only: partials stay indexed by segment and the
   * fix-up sums them in row order, so every result is bit-identical for any order.
   * kgat_csr_seg_order() builds the XCD-grouped column-sorted order. */
  const int32_t *seg_order;
} kgat_csr;

const char *kgat_strerror(int status);
int kgat_version(void);

/* Host helper: count (n_long, n_seg) for a CSR row-pointer array held in host
 * memory, then fill the plan arrays (host memory, copied to device by the
 * caller).  Pass null outputs to only count. */
int kgat_csr_plan(const int64_t *rowptr_host, int64_t n_rows, int32_t long_threshold, int32_t seg_len,
                  int32_t *n_long, int32_t *n_seg, int32_t *long_rows, int32_t *long_seg_off,
                  int32_t *seg_row, int64_t *seg_beg);

/* Host helper: the SpMM's long-row plan with column-aware cuts (host arrays).  A
 * row of degree > long_threshold is cut where a segment reaches seg_len entries, or
 * where its column crosses a multiple of col_block once the segment holds min_piece
 * entries, so a hub row's segments each gather from one slice of the source table.
 * Segments still tile each long row in order (the SpMM reads a segment's end from
 * the next segment's start).  Same outputs and count-only mode as kgat_csr_plan;
 * col_block = INT32_MAX gives kgat_csr_plan's plan. */
int kgat_csr_plan_cols(const int64_t *rowptr, const int32_t *col, int64_t n_rows, int32_t long_threshold,
                       int32_t seg_len, int32_t col_block, int32_t min_piece, int32_t *n_long, int32_t *n_seg,
                       int32_t *long_rows, int32_t *long_seg_off, int32_t *seg_row, int64_t *seg_beg);

/* Host helper: the launch order of a plan's segments for kgat_csr::seg_order
 * (host arrays; order holds 4 * ceil(n_seg / 4) entries): segments stable-sorted
 * by their first column, dealt so the long-row blocks sharing an XCD take one
 * contiguous run of that list. */
int kgat_csr_seg_order(const int32_t *col, const int64_t *seg_beg, int32_t n_seg, int32_t *order);

/* a1 -- attentive propagation SpMM, Y = A . X (+ Y when accumulate != 0).
 * Replaces torch.matmul(sparse attentive_matrix, ego_embeddings) at
 * src/model/KGAT/aggregator.py:54 and, called with the transposed CSR, its
 * autograd backward A^T . G.  d in {16, 32, 64, 128, 256}.  workspace holds
 * n_seg * d floats (partial sums of long-row segments). */
int kgat_spmm_csr_f32(const kgat_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy, int32_t d,
                      int32_t accumulate, float *workspace, int64_t workspace_floats, void *stream);

/* a1 backward restricted to a frontier (the last layer's A^T . dS, whose dS is
 * nonzero only on the <= 3*batch rows of the BPR batch):
 *   Y[r] = sum_{(r,c) in A, src_map[c] >= 0} A[r,c] Xc[src_map[c]]
 *          + (Yc_init && src_map[r] >= 0 ? Yc_init[src_map[r]] : 0)
 * src_map: int32 [n_rows] node -> compact row or -1.  Equal (up to fp32 order)
 * to the dense product with zero rows outside the frontier. */
int kgat_spmm_csr_masked_f32(const kgat_csr *A, const int32_t *src_map, const float *Xc, int64_t ldxc,
                             const float *Yc_init, int64_t ldyc, float *Y, int64_t ldy, int32_t d,
                             float *workspace, int64_t workspace_floats, void *stream);

/* The masked product of the backward's hop chain (layers below the last, whose
 * upstream gradient is nonzero only on the rows the previous A^T product
 * reached -- model.py:124-140's autograd through aggregator.py:54):
 * as kgat_spmm_csr_masked_f32, plus
 *   yc_row0: A is a row-block view whose local row r is global row yc_row0 + r
 *            (Yc_init is looked up through src_map[yc_row0 + r]);
 *   row_hit (nullable, int32 [n_rows]): zeroed, then 1 for every output row
 *            that gathered at least one frontier edge or has a Yc_init row,
 *            i.e. a superset of the rows of Y that can be nonzero;
 *   src_bits (nullable): kgat_map_bits(src_map) -- the membership test reads
 *            one bit per edge instead of a map entry;
 *   src_rank (nullable; for a src_map that numbers its set in ascending node
 *            order, e.g. kgat_hop_compact's): kgat_map_rank(src_map) -- one
 *            8-byte load per edge gives membership and compact row;
 *   n_src:   the number of source nodes (columns of A, entries of src_map;
 *            0 = unknown), reserved for a staged source set. */
int kgat_spmm_csr_masked_ex_f32(const kgat_csr *A, const int32_t *src_map, const float *Xc, int64_t ldxc,
                                const float *Yc_init, int64_t ldyc, int64_t yc_row0, float *Y, int64_t ldy,
                                int32_t d, int32_t *row_hit, const uint32_t *src_bits, const uint64_t *src_rank,
                                int64_t n_src, float *workspace, int64_t workspace_floats, void *stream);

/* The layer-0 masked product fused with the table's Adam step: the product's
 * row r (kgat_spmm_csr_masked_ex_f32 with yc_row0 = 0, no row_hit) is the
 * gradient of table row r, and instead of being written it is consumed by
 * r's Adam update (kgat_adam_f32's arithmetic, same bits) of p / m / v
 * ([n_rows x d] rows of stride ldp).  Replaces the sequence autograd
 * backward of src/model/KGAT/aggregator.py:54 into the embedding table
 * (model.py:188) + torch.optim.Adam.step() (model.py:404-413) for that
 * table: the dense gradient never reaches HBM. */
int kgat_spmm_csr_masked_adam_f32(const kgat_csr *A, const int32_t *src_map, const float *Xc, int64_t ldxc,
                                  const float *Yc_init, int64_t ldyc, const uint64_t *src_rank, float *p, float *m,
                                  float *v, int64_t ldp, int32_t d, float step_size, float beta1, float beta2,
                                  float bc2_sqrt, float eps, float *workspace, int64_t workspace_floats,
                                  void *stream);
/* ... with a skip flag (device int32, nullable): *skip != 0 when the kernel runs -> p / m / v are
 * left untouched (kgat_ids_check_ex's bad_dev: the step's ids were out of range). */
int kgat_spmm_csr_masked_adam_ex_f32(const kgat_csr *A, const int32_t *src_map, const float *Xc, int64_t ldxc,
                                     const float *Yc_init, int64_t ldyc, const uint64_t *src_rank, float *p,
                                     float *m, float *v, int64_t ldp, int32_t d, float step_size, float beta1,
                                     float beta2, float bc2_sqrt, float eps, const int32_t *skip, float *workspace,
                                     int64_t workspace_floats, void *stream);

/* kgat_spmm_csr_masked_adam_ex_f32 on a row block of a square matrix: A's row r is row yc_row0 + r
 * of the whole (the Yc_init lookup is Yc_init[src_map[yc_row0 + r]]; src_map covers the whole
 * matrix), p / m / v the block's own rows.  The row-sharded model's table update: its rows of A^T,
 * global column ids, the gathered compact [dS | dXd] rows. */
int kgat_spmm_csr_masked_adam_block_f32(const kgat_csr *A, const int32_t *src_map, const float *Xc, int64_t ldxc,
                                        const float *Yc_init, int64_t ldyc, int64_t yc_row0,
                                        const uint64_t *src_rank, float *p, float *m, float *v, int64_t ldp,
                                        int32_t d, float step_size, float beta1, float beta2, float bc2_sqrt,
                                        float eps, const int32_t *skip, float *workspace, int64_t workspace_floats,
                                        void *stream);

/* bits (uint32 [2 * ceil(n / 64)], 8-byte aligned): bit i set <=> node_map[i] >= 0. */
int kgat_map_bits(const int32_t *node_map, int64_t n, uint32_t *bits, void *stream);

/* rank (uint64 [ceil(n / 32)]): word w = (node_map of its first member) << 32 |
 * membership bits of nodes 32w .. 32w+31.  For maps numbering their set in
 * ascending node order the compact row of member c is hi + popcount(lower bits). */
int kgat_map_rank(const int32_t *node_map, int64_t n, uint64_t *rank, void *stream);

/* The next hop set from row_hit (int32 [n], 0/1): node_map[i] = position of i
 * among the flagged nodes (ascending node order) or -1, rows[0..count) = the
 * flagged nodes, *count (device int32) = their number; count_host (nullable: host-mapped
 * pinned memory, e.g. hipHostMalloc) gets the same value from the kernel, with no copy launch.
 * work: scan scratch of kgat_hop_compact_work_bytes(n) bytes. */
int64_t kgat_hop_compact_work_bytes(int64_t n);
int kgat_hop_compact(const int32_t *hit, int64_t n, int32_t *node_map, int32_t *rows, int32_t *count,
                     int32_t *count_host, void *work, int64_t work_bytes, void *stream);

/* The first hop of the backward chain without scanning the graph: for the
 * last layer's A^T product over the batch frontier F (rows0[0..n0), -1
 * padded, kgat_frontier_build), bits0 (uint32 [ceil(n/32)]) marks F and
 * bits1 marks F plus every column of A's rows F -- the rows that product can
 * reach; node_map / hop_rows / *hop_count list bits1's set in ascending node
 * order (node_map fully written, -1 outside); hop_count_host (nullable) as kgat_hop_compact's
 * count_host; hop_rank (nullable, uint64
 * [ceil(n/32)]) gets the set's rank words (kgat_map_rank's layout).  work:
 * kgat_frontier_hop_work_bytes(n) bytes (8-byte aligned), zero-filled before
 * its first use; every call leaves it reusable (it holds the single-pass
 * scan's state: one call at a time per work buffer, stream-ordered). */
int64_t kgat_frontier_hop_work_bytes(int64_t n);
int kgat_frontier_hop(const kgat_csr *A, const int32_t *rows0, int32_t n0, uint32_t *bits0, uint32_t *bits1,
                      int32_t *node_map, int32_t *hop_rows, int32_t *hop_count, int32_t *hop_count_host,
                      uint64_t *hop_rank, void *work, int64_t work_bytes, void *stream);
/* flags: KGAT_HOP_PRECLEARED -- bits0 / bits1 are already zero (kgat_cf_begin cleared them): the
 * clearing launch is skipped. */
#define KGAT_HOP_PRECLEARED 1
int kgat_frontier_hop_ex(const kgat_csr *A, const int32_t *rows0, int32_t n0, uint32_t *bits0, uint32_t *bits1,
                         int32_t *node_map, int32_t *hop_rows, int32_t *hop_count, int32_t *hop_count_host,
                         uint64_t *hop_rank, void *work, int64_t work_bytes, int32_t flags, void *stream);

/* kgat_spmm_csr_masked_f32 restricted to an output row set (A = A^T of the
 * graph; out_bits / out_map / out_rows / out_count from kgat_frontier_hop):
 * Y[k] = row out_rows[k] of the masked product, for k < *out_count (compact,
 * Y holds n_rows rows of capacity); rows outside the set are not visited.
 * src_bits (nullable) = the source set's bitmap.  Per row the same edges in
 * the same order as the dense masked product (same bits). */
int kgat_spmm_csr_masked_rows_f32(const kgat_csr *A, const int32_t *src_map, const uint32_t *src_bits,
                                  const float *Xc, int64_t ldxc, const float *Yc_init, int64_t ldyc,
                                  const uint32_t *out_bits, const int32_t *out_map, const int32_t *out_rows,
                                  const int32_t *out_count, float *Y, int64_t ldy, int32_t d, float *workspace,
                                  int64_t workspace_floats, void *stream);
/* ... plus Gc (nullable, ldgc): compact rows added to Y[k] after the Yc_init term through the same
 * src_map row -- the BPR loss's direct gradient of the batch rows (kgat_bpr_bwd_multi_f32), i.e.
 * kgat_bpr_bwd_f32 into Y with row_map = out_map folded into this launch (same bits); out_src
 * (nullable, int32 [n_rows]): out_src[k] = src_map[out_rows[k]] for k < *out_count (the compact source
 * row of output row k, -1 = none: kgat_biinter_bwd_hop_ex_f32's gidx). */
int kgat_spmm_csr_masked_rows_ex_f32(const kgat_csr *A, const int32_t *src_map, const uint32_t *src_bits,
                                     const float *Xc, int64_t ldxc, const float *Yc_init, int64_t ldyc,
                                     const float *Gc, int64_t ldgc, const uint32_t *out_bits, const int32_t *out_map,
                                     const int32_t *out_rows, const int32_t *out_count, float *Y, int64_t ldy,
                                     int32_t *out_src, int32_t d, float *workspace, int64_t workspace_floats,
                                     void *stream);

/* Rows of A that are in a node set or have an edge into it: hit[r] = 1 iff bit (row0 + r) of
 * bits or bit col of one of row r's edges is set, else 0 (n_bits: the bitmap's size in nodes,
 * covering every column and row0 + n_rows).  With A = a shard's rows of A^T and the bitmap of
 * the batch rows F, the shard's part of the first hop F + N(F) (A^T[j, f] != 0 <=> A[f, j] != 0):
 * the row set the row-sharded frontier forward computes layer L-2 on.  Long rows are scanned by
 * their segments (A's long-row plan). */
int kgat_csr_mark_rows(const kgat_csr *A, const uint32_t *bits, int64_t n_bits, int64_t row0, int32_t *hit,
                       void *stream);

/* The forward restricted to a hop set (KGAT.frontier_forward; the row set a
 * training step's loss can reach, see model._CFLoss): the dense product
 * Y[r] = (A . X)[r] for the rows r of an output set only -- out_rows[k] for
 * k < *out_count (device; each in [0, n_rows) or -1, which is skipped), out_bits its bitmap --,
 * each written at its own row of Y (other rows untouched).  Per row the same
 * edges in the same order as kgat_spmm_csr_f32 (same bits).  Replaces
 * aggregator.py:54's product on the rows model.py:189-191 gathers from. */
int kgat_spmm_csr_rows_f32(const kgat_csr *A, const float *X, int64_t ldx, const uint32_t *out_bits,
                           const int32_t *out_rows, const int32_t *out_count, float *Y, int64_t ldy, int32_t d,
                           float *workspace, int64_t workspace_floats, void *stream);

/* Data-parallel exchange of the compact table gradient (replicas.ShardedGradSync,
 * replicate_table mode; no reference counterpart -- the reference is one
 * process).  Every replica's layer-0 hop set is an ascending row list; after an
 * all-gather, list g = lists[g*cap .. g*cap + counts[g]) (counts on the device).
 * kgat_rows_union: their union, as kgat_frontier_hop's outputs (bits uint32
 * [ceil(n/32)], node_map, rows, *count, rank words; work:
 * kgat_frontier_hop_work_bytes(n)).  kgat_rows_merge_f32: for k < *count
 * (<= max_rows), out[k] = scale * sum over g (in g order) of the row of vals
 * (w floats, row g*cap + position of rows[k] in list g) of every list holding
 * rows[k]; G <= 64, w and the leading dimensions multiples of 4. */
int kgat_rows_union(const int32_t *lists, const int32_t *counts, int32_t G, int32_t cap, int64_t n, uint32_t *bits,
                    int32_t *node_map, int32_t *rows, int32_t *count, uint64_t *rank, void *work, int64_t work_bytes,
                    void *stream);
int kgat_rows_merge_f32(const int32_t *lists, const int32_t *counts, int32_t G, int32_t cap, const float *vals,
                        int64_t ldv, int32_t w, const int32_t *rows, const int32_t *count, int64_t max_rows,
                        float *out, int64_t ldo, float scale, void *stream);

/* a2 -- bi-interaction aggregator forward, fused:
 *   H = normalize(dropout(LReLU(W1 (X+S) + b1) + LReLU(W2 (X*S) + b2)))
 * Replaces src/model/KGAT/aggregator.py:57-65.  W1/W2 are nn.Linear weights
 * [d_out, d_in].  dropout_p in [0,1); the keep mask is a counter hash of
 * (seed, row, column), regenerated by the backward.  d_in, d_out in
 * {16, 32, 64, 128}.
 * norm_out / mask_out (both or neither): the saved state the backward uses
 * instead of recomputing the forward -- norm_out float [n_rows] (the row L2
 * norm, -eps where F.normalize's clamp was active) and mask_out uint64
 * [ceil(n_rows/16) * NG * 64], NG = ceil(d_out/64) (per 16-row sub-tile st,
 * word group g = 16-column block / 4 and lane: word (st*NG + g)*64 + lane
 * holds 3 bits per output element -- pre_sum > 0, pre_mul > 0, dropout keep).
 * d_out <= 64 (NG = 1) feeds kgat_biinter_bwd_f32 / _hop_f32; d_out = 128
 * feeds kgat_biinter_bwd_gemm_bits_f32 (then node0 = 0). */
int kgat_biinter_fwd_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *W1,
                         const float *b1, const float *W2, const float *b2, float *H, int64_t ldh,
                         int64_t n_rows, int32_t d_in, int32_t d_out, float dropout_p, uint64_t seed,
                         float *norm_out, uint64_t *mask_out, void *stream);

/* kgat_biinter_fwd_f32 on the 16-row tiles of the table holding a member of
 * the node set row_bits (uint32 bitmap [ceil(n_rows/32)], e.g. a hop set of
 * kgat_frontier_hop) only: H, norm_out and mask_out of those tiles are written
 * exactly as the whole-table call writes them, the rest is untouched.
 * aggregator.py:57-65 on a hop set. */
int kgat_biinter_fwd_tiles_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *W1,
                               const float *b1, const float *W2, const float *b2, float *H, int64_t ldh,
                               int64_t n_rows, const uint32_t *row_bits, int32_t d_in, int32_t d_out,
                               float dropout_p, uint64_t seed, float *norm_out, uint64_t *mask_out, void *stream);

/* kgat_biinter_fwd_f32 on the 4-row quads (rows 4k .. 4k+3) holding a listed
 * node: rows[0 .. *count) (int32, device count, read as at most cap; -1 =
 * padding; cap = the list's capacity, which also bounds the grid), e.g. the ascending row list of a
 * hop set (kgat_frontier_hop) or the batch rows (kgat_cf_begin_ex).  H,
 * norm_out and the state words of those quads are written exactly as the
 * whole-table call writes them (a quad listed twice is written twice with the
 * same bits), the rest is untouched.  aggregator.py:57-65 on a row set. */
int kgat_biinter_fwd_list_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *W1,
                              const float *b1, const float *W2, const float *b2, float *H, int64_t ldh,
                              int64_t n_rows, const int32_t *rows, const int32_t *count, int64_t cap,
                              int32_t d_in, int32_t d_out, float dropout_p, uint64_t seed, float *norm_out,
                              uint64_t *mask_out, void *stream);

/* kgat_biinter_fwd_f32 on rows [node0, node0 + n_rows) of a larger table: X, S,
 * H, norm_out, mask_out point at that block's first row (mask_out at word
 * (node0 / 16) * 64), the dropout draws use the global node ids.  node0 a
 * multiple of 16.  Lets the forward run the bi-interaction of row block b
 * (one stream) while the propagation of block b + 1 runs (another stream). */
int kgat_biinter_fwd_rows_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *W1,
                              const float *b1, const float *W2, const float *b2, float *H, int64_t ldh,
                              int64_t n_rows, int64_t node0, int32_t d_in, int32_t d_out, float dropout_p,
                              uint64_t seed, float *norm_out, uint64_t *mask_out, void *stream);

/* Workspace (floats) kgat_biinter_bwd_f32 needs for its weight-gradient slabs. */
int64_t kgat_biinter_bwd_workspace(int64_t n_rows, int32_t d_in, int32_t d_out);

/* a2 backward (autograd of aggregator.py:57-65): given dH, writes
 *   dXd = d/dX through the bi-interaction (direct path) and dS = d/dS,
 * and dW1, db1, dW2, db2 (overwritten, deterministic slab reduction).
 * rows (nullable, int32 [n_rows]): frontier mode -- compact row i of dH / dXd
 * / dS belongs to node rows[i] of X and S (src_rows rows; -1 = padding).
 * H / norm / mask (all or none): the forward's output and saved state (indexed
 * by node like X); given, nothing of the forward is recomputed (d_out <= 64 and
 * d_in * d_out <= 4096), otherwise the forward is recomputed from X, S, W, b. */
int kgat_biinter_bwd_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *H,
                         int64_t ldh, const float *norm, const uint64_t *mask, const float *dH,
                         int64_t lddh, const float *W1, const float *b1, const float *W2, const float *b2,
                         float *dXd, int64_t lddxd, float *dS, int64_t ldds, float *dW1, float *db1,
                         float *dW2, float *db2, int64_t n_rows, int32_t d_in, int32_t d_out,
                         float dropout_p, uint64_t seed, const int32_t *rows, int64_t src_rows,
                         float *workspace, int64_t workspace_floats, void *stream);

/* a2 backward on a hop set of the backward chain (see kgat_hop_compact /
 * kgat_frontier_hop): rows / count are that call's outputs (count stays on the
 * device; n_max bounds it); dH is indexed by node like X (the dense output of
 * the previous masked product) or, with dh_compact, by hop position (row i of
 * dH <-> node rows[i], kgat_spmm_csr_masked_rows_f32's output); dXd / dS are
 * compact (n_max rows allocated).  Saved forward state only (H, norm, mask;
 * d_out <= 64 and d_in * d_out <= 4096).  Per row the arithmetic is
 * kgat_biinter_bwd_f32's. */
int kgat_biinter_bwd_hop_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *H, int64_t ldh,
                             const float *norm, const uint64_t *mask, const float *dH, int64_t lddh,
                             const float *W1, const float *W2, float *dXd, int64_t lddxd, float *dS, int64_t ldds,
                             float *dW1, float *db1, float *dW2, float *db2, const int32_t *rows,
                             const int32_t *count, int64_t n_max, int64_t src_rows, int32_t dh_compact,
                             int32_t d_in, int32_t d_out, float dropout_p, float *workspace,
                             int64_t workspace_floats, void *stream);
/* ... plus the BPR term of the batch rows: G (nullable, ldg >= d_in) holds compact rows and gidx (int32,
 * with G; by hop position, e.g. kgat_spmm_csr_masked_rows_ex_f32's out_src) names the G row of hop row i
 * or -1.  Hop row i with gidx[i] >= 0 gets dXd += G[gidx[i]] after its bi-interaction term
 * (kgat_bpr_bwd_f32 into dXd with row_map = the hop map, folded in: same bits).  gmap (nullable): the
 * batch-row node map that numbers G; its entries of those rows are reset to -1 by the same launch
 * (kgat_frontier_reset folded in: rows must hold every node gmap numbers). */
int kgat_biinter_bwd_hop_ex_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *H, int64_t ldh,
                                const float *norm, const uint64_t *mask, const float *dH, int64_t lddh,
                                const float *W1, const float *W2, float *dXd, int64_t lddxd, float *dS, int64_t ldds,
                                float *dW1, float *db1, float *dW2, float *db2, const int32_t *rows,
                                const int32_t *count, int64_t n_max, int64_t src_rows, int32_t dh_compact,
                                int32_t d_in, int32_t d_out, float dropout_p, const float *G, int64_t ldg,
                                const int32_t *gidx, int32_t *gmap, float *workspace, int64_t workspace_floats,
                                void *stream);

/* The dense fp32 contractions of the wide layers (a2 / a6 at d = 128 / 256: W1, W2,
 * W_r, W_v, W_o products and the split-K weight-gradient slabs), hand-written MFMA
 * (v_mfma_f32_32x32x2_f32, 128 x 128 block tiles, deterministic k order):
 *   C[m, n] (+)= sum_k op(A)[m, k] op(B)[k, n], row-major;
 *   op(A) = A [m, k] (lda) or, trans_a, A^T of A stored [k, m];
 *   op(B) = B [k, n] (ldb) or, trans_b, B^T of B stored [n, k];
 *   batch z: A + z*stride_a, B + z*stride_b, C + z*stride_c.
 * lda, ldb, strides and bases 16-byte aligned; each operand's contiguous dimension a
 * multiple of 4.  Replaces the vendor sgemm a torch port would call for
 * nn.Linear at aggregator.py:57-60 and the bmm / Linear of model.py:271-303. */
int kgat_gemm_f32(int32_t trans_a, int32_t trans_b, int64_t m, int64_t n, int64_t k, const float *A, int64_t lda,
                  int64_t stride_a, const float *B, int64_t ldb, int64_t stride_b, float *C, int64_t ldc,
                  int64_t stride_c, int64_t batch, int32_t accumulate, void *stream);

/* a2 for the wide layers of C4/C5 (any d_in, d_out multiple of 16 up to 1024; used
 * where the fused kernels above do not dispatch, e.g. 256): two kgat_gemm_f32 products
 * per direction around fused HIP epilogues, same arithmetic and the same dropout
 * draws as kgat_biinter_fwd_f32.
 * state (float [kgat_biinter_gemm_state_floats]) is written by the forward
 * (pre-activations + row norms) and consumed (overwritten) by the backward;
 * work (float [kgat_biinter_gemm_work_floats]) is scratch for either call.
 * key_rows (nullable): the node id of each row for the dropout draws when the
 * rows are a gathered frontier (-1 = padding row: zero gradient). */
int64_t kgat_biinter_gemm_state_floats(int64_t n_rows, int32_t d_in, int32_t d_out);
int64_t kgat_biinter_gemm_work_floats(int64_t n_rows, int32_t d_in, int32_t d_out);
int kgat_biinter_fwd_gemm_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *W1,
                              const float *b1, const float *W2, const float *b2, float *H, int64_t ldh,
                              int64_t n_rows, int32_t d_in, int32_t d_out, float dropout_p, uint64_t seed,
                              float *state, float *work, int64_t work_floats, void *stream);
/* The GEMM forward on the rows rows[0..m) of X / S only (node ids in [0, n_rows), -1 = padding,
 * skipped): each listed row's H row, state (pre-activations, norm) and dropout draws land at its
 * own index, bit for bit the whole-table call's; other rows are untouched.  The row-sharded
 * frontier forward of a wide layer on the first hop.  work: kgat_biinter_gemm_rows_work_floats(m). */
int64_t kgat_biinter_gemm_rows_work_floats(int64_t m, int32_t d_in, int32_t d_out);
int kgat_biinter_fwd_gemm_rows_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const int32_t *rows,
                                   int64_t m, const float *W1, const float *b1, const float *W2, const float *b2,
                                   float *H, int64_t ldh, int64_t n_rows, int32_t d_in, int32_t d_out,
                                   float dropout_p, uint64_t seed, float *state, float *work, int64_t work_floats,
                                   void *stream);
int kgat_biinter_bwd_gemm_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *H,
                              int64_t ldh, float *state, const float *dH, int64_t lddh, const float *W1,
                              const float *W2, float *dXd, int64_t lddxd, float *dS, int64_t ldds, float *dW1,
                              float *db1, float *dW2, float *db2, int64_t n_rows, int32_t d_in, int32_t d_out,
                              float dropout_p, uint64_t seed, const int32_t *key_rows, float *work,
                              int64_t work_floats, void *stream);
/* The same backward from the fused forward's saved state (kgat_biinter_fwd_f32's
 * norm_out / mask_out, d_out <= 128, indexed by node = key_rows[i] or i) instead of
 * pre-activations: C4's 128 -> 128 / 128 -> 64 layers run the fused MFMA forward
 * (no [n, 2*d_out] pre-activation state written) and this GEMM backward.
 * work: float [kgat_biinter_gemm_bits_work_floats]. */
int64_t kgat_biinter_gemm_bits_work_floats(int64_t n_rows, int32_t d_in, int32_t d_out);

/* The wide backward on the rows rows[0..m) of a layer only (the hop rows of the backward chain),
 * without gathering them: X, S, H, dH (all [n_rows, *], indexed by node) and the forward's state
 * are read at each listed node's own row, dXd / dS [m, d_in] are written compactly (row r = node
 * rows[r]; -1 = padding, zero), the weight gradients sum the listed rows -- the same bits as the
 * gathered compact call (kgat_biinter_bwd_gemm_f32 / _bits_f32 with key_rows on gathered rows).
 * state: the GEMM forward's pre-activations + norms (norm, mask null), or null with the fused
 * forward's norm + mask words (d_out <= 128).  work: kgat_biinter_bwd_gemm_rows_work_floats(m). */
int64_t kgat_biinter_bwd_gemm_rows_work_floats(int64_t m, int32_t d_in, int32_t d_out);
int kgat_biinter_bwd_gemm_rows_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *H,
                                   int64_t ldh, const float *state, const float *norm, const uint64_t *mask,
                                   const float *dH, int64_t lddh, const int32_t *rows, int64_t m, const float *W1,
                                   const float *W2, float *dXd, int64_t lddxd, float *dS, int64_t ldds, float *dW1,
                                   float *db1, float *dW2, float *db2, int64_t n_rows, int32_t d_in, int32_t d_out,
                                   float dropout_p, uint64_t seed, float *work, int64_t work_floats, void *stream);
/* ... in two calls on the same work buffer: phases 1 = the operand gathers, the epilogue and the
 * dXd / dS GEMM; phases 2 = the weight gradients (reads what phase 1 left in work); 3 = both.  The
 * row-sharded backward posts dS / dXd to its peers between the two, so the weight-gradient GEMMs run
 * under that gather.  Same bits as one call. */
int kgat_biinter_bwd_gemm_rows_ex_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *H,
                                      int64_t ldh, const float *state, const float *norm, const uint64_t *mask,
                                      const float *dH, int64_t lddh, const int32_t *rows, int64_t m, const float *W1,
                                      const float *W2, float *dXd, int64_t lddxd, float *dS, int64_t ldds,
                                      float *dW1, float *db1, float *dW2, float *db2, int64_t n_rows, int32_t d_in,
                                      int32_t d_out, float dropout_p, uint64_t seed, float *work,
                                      int64_t work_floats, int32_t phases, void *stream);
int kgat_biinter_bwd_gemm_bits_f32(const float *X, int64_t ldx, const float *S, int64_t lds, const float *H,
                                   int64_t ldh, const float *norm, const uint64_t *mask, const float *dH,
                                   int64_t lddh, const float *W1, const float *W2, float *dXd, int64_t lddxd,
                                   float *dS, int64_t ldds, float *dW1, float *db1, float *dW2, float *db2,
                                   int64_t n_rows, int32_t d_in, int32_t d_out, float dropout_p,
                                   const int32_t *key_rows, float *work, int64_t work_floats, void *stream);

/* §8(f)2 -- CF / KG batch samplers (host, src/model/KGAT/preprocess.py:328-525).
 * CF: `batch` users from users[0..n_users) (distinct when batch <= n_users, in random
 *   order), for each one positive uniform over items[rowptr[k]..rowptr[k+1]) (sorted,
 *   unique) and one negative uniform over [0, item_num) not among them.
 * KG: `batch` heads from heads[0..n_heads) likewise; rel_tail[rowptr[k]..rowptr[k+1])
 *   holds relation * n_nodes + tail, sorted; one positive (relation, tail) uniform over
 *   them and one negative tail uniform over [0, n_nodes) with (head, relation, tail)
 *   not an edge.  Random numbers: splitmix64 of (seed, step, draw) -- reproducible. */
int kgat_sample_cf_batch(const int64_t *users, int64_t n_users, const int64_t *rowptr, const int64_t *items,
                         int64_t item_num, int32_t batch, uint64_t seed, uint64_t step, int64_t *out_users,
                         int64_t *out_pos, int64_t *out_neg);
int kgat_sample_kg_batch(const int64_t *heads, int64_t n_heads, const int64_t *rowptr, const int64_t *rel_tail,
                         int64_t n_nodes, int32_t batch, uint64_t seed, uint64_t step, int64_t *out_heads,
                         int64_t *out_rels, int64_t *out_pos, int64_t *out_neg);

/* §8(f)2 -- NFM feature batches (NFM/preprocess.py:150-193, 309-356): row r =
 * [one-hot user u_r | feature row of item i_r] over user_num + entity_num columns,
 * from the item feature CSR (feat_rowptr/feat_col/feat_val, item_num rows).
 * items == NULL: the test-batch grid, row r = (users[r / item_num], r % item_num).
 * kgat_nfm_batch_rowptr writes rowptr_out [rows + 1] (device); the caller reads
 * rowptr_out[rows] (= nnz), sizes the outputs and calls kgat_nfm_batch_fill, which
 * writes each row's entries, user column first, then the feature row's columns
 * shifted by user_num (row_out, optional, = the COO row of each entry). */
int64_t kgat_nfm_batch_work_bytes(int64_t rows);
int kgat_nfm_batch_rowptr(const int64_t *users, const int64_t *items, int64_t rows, int64_t item_num,
                          const int64_t *feat_rowptr, int64_t *rowptr_out, void *work, int64_t work_bytes,
                          void *stream);
int kgat_nfm_batch_fill(const int64_t *users, const int64_t *items, int64_t rows, int64_t item_num,
                        int64_t user_num, const int64_t *feat_rowptr, const int64_t *feat_col,
                        const float *feat_val, const int64_t *rowptr, int64_t *row_out, int64_t *col_out,
                        float *val_out, void *stream);

/* Tables of a propagated embedding: [X0 | H1 | ... | HL] kept as separate
 * row-major buffers (the reference torch.cat's them, model.py:140). */
#define KGAT_MAX_TABLES 8
typedef struct kgat_tables {
  const float *ptr[KGAT_MAX_TABLES];
  int64_t ld[KGAT_MAX_TABLES];
  int32_t width[KGAT_MAX_TABLES];
  int32_t count;
} kgat_tables;

/* a3/a4 -- CF BPR loss forward (model.py:165-202): gathers user/pos/neg rows
 * (item ids index the table raw, model.py:189-191), writes the scalar loss and
 * per-sample coefficients coef[b] = sigmoid(pos_b - neg_b) - 1 for the
 * backward.  ids are int64 [batch]; coef holds 2*batch floats (the second
 * half keeps the per-sample loss terms, summed in index order). */
int kgat_bpr_fwd_f32(const kgat_tables *T, const int64_t *users, const int64_t *pos, const int64_t *neg,
                     int32_t batch, float reg, float *loss, float *coef, void *stream);
/* ... in one launch: ticket (nullable; device uint32, 0 on entry, left 0) -- the block that finishes
 * last sums the loss terms (same order, same bits as the second kernel of kgat_bpr_fwd_f32).  Calls
 * sharing a ticket must be stream-ordered. */
int kgat_bpr_fwd_ex_f32(const kgat_tables *T, const int64_t *users, const int64_t *pos, const int64_t *neg,
                        int32_t batch, float reg, float *loss, float *coef, uint32_t *ticket, void *stream);

/* a3/a4 backward: for table t, dst[id] += d loss / d table_t[id] for every
 * gathered id, duplicates summed in slot order (deterministic).  grad_out
 * points at the scalar upstream gradient (device).  row_map (nullable): write
 * to dst row row_map[id] instead of id (compact frontier rows); ids with
 * row_map[id] < 0 are skipped (rows another shard owns). */
int kgat_bpr_bwd_f32(const kgat_tables *T, int32_t table, const int64_t *users, const int64_t *pos,
                     const int64_t *neg, int32_t batch, float reg, const float *coef,
                     const float *grad_out, float *dst, int64_t lddst, const int32_t *row_map, void *stream);
/* kgat_bpr_bwd_f32 for tables t0 .. T->count - 1 in one launch, each WRITTEN (not added) into its
 * own compact buffer D->ptr[t] (ld D->ld[t]; null = skip that table) at the row's frontier position
 * (rows / *count: kgat_frontier_build's list of the batch's distinct ids): the summed gradient with
 * kgat_bpr_bwd_f32's arithmetic into zeros (same bits); rows [*count, 3 * batch) of every buffer are
 * zeroed.  The backward's batch-row terms of every layer at once, consumed as the last layer's dH, by
 * kgat_spmm_csr_masked_rows_ex_f32 (Gc) and by kgat_biinter_bwd_hop_ex_f32 (G). */
int kgat_bpr_bwd_multi_f32(const kgat_tables *T, int32_t t0, const int64_t *users, const int64_t *pos,
                           const int64_t *neg, int32_t batch, float reg, const float *coef, const float *grad_out,
                           const kgat_tables *D, const int32_t *rows, const int32_t *count, void *stream);

/* The BPR batch's distinct rows (the backward frontier of the last layer,
 * model.py:189-191 gathers only these): rows[0..count) = ids in
 * first-occurrence order, node_map[id] = position, rows[count..3*batch) = -1.
 * node_map (int32 [n_nodes]) must be all -1 on entry; kgat_frontier_reset
 * restores it.  3*batch <= 4096. */
int kgat_frontier_build(const int64_t *users, const int64_t *pos, const int64_t *neg, int32_t batch,
                        int32_t *node_map, int32_t *rows, int32_t *count, void *stream);
int kgat_frontier_reset(const int32_t *rows, int32_t n, int32_t *node_map, void *stream);

/* The prologue of a TRAIN_CF step (model.py:165-202 on device ids) in one launch: kgat_ids_check_ex on
 * users | pos | neg (int64 [batch] each) against [0, bound) -- ids_out (int64 [3 * batch]) gets the
 * checked copies in that order, an id out of range becomes 0 and sets *bad (and *bad_dev when given) --,
 * kgat_frontier_build on the checked ids (node_map / rows / count), and, when clear0 / clear1 are given
 * (16-byte aligned, clear_words uint32 each), the zeroing of kgat_frontier_hop's two bitmaps
 * (then call it with KGAT_HOP_PRECLEARED).  3 * batch <= 4096. */
int kgat_cf_begin(const int64_t *users, const int64_t *pos, const int64_t *neg, int32_t batch, int64_t bound,
                  int64_t *ids_out, int32_t *bad, int32_t *bad_dev, int32_t *node_map, int32_t *rows, int32_t *count,
                  uint32_t *clear0, uint32_t *clear1, int64_t clear_words, void *stream);
/* kgat_cf_begin with a completion tag and the first hop's marking.  tag = 0: *bad as in kgat_cf_begin;
 * 0 < tag < 2^29: bad points to two words (host-mapped pinned memory), written once after the check by
 * one thread with stores through to memory: bad[0] = 1 when an id was out of range (never cleared by the
 * kernel: the caller clears it), then bad[1] = tag (a release store behind bad[0] when that was written).
 * The host polls bad[1] for its tag instead of recording an event behind the launch (an event record
 * costs ~5 us of GPU time between two dependent kernels).  mark0 / mark1 (nullable; zero on entry, a
 * different pair from clear0 / clear1, A's n_rows >= bound): the same launch marks the batch's first hop
 * there as kgat_frontier_hop does (mark0: the batch rows, mark1: those rows and every column of their
 * rows of A) -- then call kgat_frontier_hop_ex with n0 = 0 and KGAT_HOP_PRECLEARED to list it.  Clearing
 * one bitmap pair while marking the other lets a caller alternate two pairs across steps (model.py). */
int kgat_cf_begin_ex(const int64_t *users, const int64_t *pos, const int64_t *neg, int32_t batch, int64_t bound,
                     int64_t *ids_out, int32_t *bad, int32_t *bad_dev, int32_t *node_map, int32_t *rows,
                     int32_t *count, uint32_t *clear0, uint32_t *clear1, int64_t clear_words, const kgat_csr *A,
                     uint32_t *mark0, uint32_t *mark1, int32_t tag, void *stream);

/* a5 -- TransR KG loss (model.py:204-261): h' = e_h W_r etc., scalar loss
 * written to *loss.  work (kgat_transr_work_floats) keeps per-sample terms and
 * gradients for the backward.  d, k <= 256. */
int64_t kgat_transr_work_floats(int32_t batch, int32_t d, int32_t k);
int kgat_transr_fwd_f32(const float *emb, int64_t ld_emb, const float *rel_emb, const float *trans, int32_t d,
                        int32_t k, const int64_t *heads, const int64_t *rels, const int64_t *pos,
                        const int64_t *neg, int32_t batch, float reg, float *loss, float *work, void *stream);
/* a5 forward with the relation count: for d >= 128 (d, k in {128, 256} x {64, 128, 256})
 * one block per (relation, 16-sample chunk of its samples in batch order) runs both
 * products of the chunk on the fp32 MFMA with W_r read once per chunk; otherwise the
 * per-sample kernel of kgat_transr_fwd_f32.  Same work layout, same loss definition. */
int kgat_transr_fwd_ex_f32(const float *emb, int64_t ld_emb, const float *rel_emb, const float *trans, int32_t d,
                           int32_t k, int32_t n_rel, const int64_t *heads, const int64_t *rels, const int64_t *pos,
                           const int64_t *neg, int32_t batch, float reg, float *loss, float *work, void *stream);
/* a5 backward: d_emb[id] += (upstream * dL/de) for every gathered id (duplicates
 * summed in slot order; d_emb must be initialised, e.g. zero), d_rel [n_rel, k]
 * and d_trans [n_rel, d, k] overwritten: each relation's samples (batch order) are
 * cut into 32-sample chunks, one block per chunk sums its chunk in order, and the
 * chunk partials are summed in chunk order -- deterministic, balanced when a few
 * relations (the CKG's interaction pair) hold most samples.  workspace: float
 * [kgat_transr_bwd_workspace_floats(batch, d, k, n_rel)]. */
int64_t kgat_transr_bwd_workspace_floats(int32_t batch, int32_t d, int32_t k, int32_t n_rel);
int kgat_transr_bwd_f32(const float *emb, int64_t ld_emb, int32_t d, int32_t k, const int64_t *heads,
                        const int64_t *rels, const int64_t *pos, const int64_t *neg, int32_t batch, int32_t n_rel,
                        const float *work, const float *grad_out, float *d_emb, int64_t ld_demb, float *d_rel,
                        float *d_trans, float *workspace, int64_t workspace_floats, void *stream);
/* As kgat_transr_bwd_f32 with the table gradient written compactly: row row_map[id] of d_emb
 * (kgat_frontier_build's node map of the batch ids; the caller zero-fills its <= 3 * batch rows)
 * instead of row id -- the input of kgat_adam_rows_f32 (the fused KG table update). */
int kgat_transr_bwd_ex_f32(const float *emb, int64_t ld_emb, int32_t d, int32_t k, const int64_t *heads,
                           const int64_t *rels, const int64_t *pos, const int64_t *neg, int32_t batch, int32_t n_rel,
                           const float *work, const float *grad_out, float *d_emb, int64_t ld_demb,
                           const int32_t *row_map, float *d_rel, float *d_trans, float *workspace,
                           int64_t workspace_floats, void *stream);

/* a6 -- knowledge-aware edge scores (model.py:263-316, multi_head_attention.py:35-58):
 * logit_e = sum_j tanh(LN(W_o drop(W_v (e_t W_r) + b_v) + b_o))_j * edge_weight[e]
 * for edges in 16-edge single-relation tiles: tile t covers
 * rel_perm[tile_beg[t] .. tile_beg[t+1]) with relation tile_rel[t].  Query/key
 * are dead (softmax over one key == 1).  dropout_p > 0 applies the train-mode
 * per-(edge, head) attention dropout.  Output logits[out_pos[e]] (or logits[e]
 * when out_pos is null).  d in {16, 32, 64, 128}. */
int kgat_edge_logits_f32(const float *emb, int64_t ld_emb, int64_t n_nodes, const float *trans, int32_t d,
                         const float *Wv, const float *bv, const float *Wo, const float *bo, const float *ln_w,
                         const float *ln_b, const int32_t *tails, const float *edge_weight,
                         const int32_t *rel_perm, const int32_t *tile_rel, const int32_t *tile_beg,
                         int32_t n_tiles, float dropout_p, uint64_t seed, const int32_t *out_pos, float *logits,
                         void *stream);
/* Sum edge logits per CSR slot (duplicate (head, tail) pairs, model.py:359-363). */
int kgat_slot_sum_f32(const int64_t *slot_edge_ptr, const int32_t *edge_order, int64_t nnz,
                      const float *edge_logits, float *slot_logits, void *stream);
/* a7 -- val = row softmax over the stored entries (torch.sparse.softmax(dim=1), model.py:364). */
int kgat_row_softmax_f32(const int64_t *rowptr, int64_t n_rows, const float *slot_logits, float *val,
                         void *stream);
/* kgat_row_softmax_f32 with the rows of more than 256 entries listed
 * (long_rows[0..n_long), e.g. the CSR's long-row plan at threshold 256): those
 * take a block each, the others 4- or 16-lane groups with the row in registers.
 * long_rows == NULL: the long rows are found by a scan of all rows. */
int kgat_row_softmax_ex_f32(const int64_t *rowptr, int64_t n_rows, const int32_t *long_rows, int32_t n_long,
                            const float *slot_logits, float *val, void *stream);
/* a7 with the CSR's long-row plan (seg_len 512, long_threshold 256, as kgat_csr_plan's defaults): rows of
 * <= 256 entries 16 per wave, by length class (<= 8 and <= 32 entries: a 4-lane group, 2 / 8 entries per
 * lane; 33..256: a 16-lane group, 16 per lane); a longer row is cut into its plan segments -- pass 1 keeps
 * each segment's max and sum of exp (work: kgat_row_softmax_work_floats(A) floats), pass 2 combines the
 * row's segments in segment order (max, then the rescaled sums) and every segment writes its entries.
 * A row's values depend on its entries only (the same bits in a row view or a shard). */
int64_t kgat_row_softmax_work_floats(const kgat_csr *A);
int kgat_row_softmax_plan_f32(const kgat_csr *A, const float *slot_logits, float *val, float *work,
                              int64_t work_floats, void *stream);

/* a6 for wide embeddings (d > 128, multiple of 16, <= 1024; C5's 256): the edge scorer
 * of kgat_edge_logits_f32 as kgat_gemm_f32 products over chunks of the relation-sorted edge
 * order plus fused HIP epilogues -- same arithmetic, dropout keys and output placement.
 * seg_rel / seg_beg (HOST arrays): relation of each run of rel_perm and the runs'
 * start positions (n_seg + 1 entries, last = n_edges).  work: float
 * [kgat_edge_logits_gemm_work_floats(chunk, d)] for chunks of `chunk` edges. */
int64_t kgat_edge_logits_gemm_work_floats(int64_t chunk_edges, int32_t d);
int kgat_edge_logits_gemm_f32(const float *emb, int64_t ld_emb, int64_t n_nodes, const float *trans, int32_t d,
                              const float *Wv, const float *bv, const float *Wo, const float *bo, const float *ln_w,
                              const float *ln_b, const int32_t *tails, const float *edge_weight,
                              const int32_t *rel_perm, int64_t n_edges, const int32_t *seg_rel,
                              const int64_t *seg_beg, int32_t n_seg, float dropout_p, uint64_t seed,
                              const int32_t *out_pos, float *out, float *work, int64_t work_floats, void *stream);

/* a8 -- CF scores (model.py:368-391): scores[u, i] = <all[users[u]], all[items[i]]>
 * over the concatenated tables (row-major [n_users, ld_scores]).  Table widths
 * must be multiples of 16. */
int kgat_score_f32(const kgat_tables *T, const int64_t *users, int32_t n_users, const int64_t *items,
                   int32_t n_items, float *scores, int64_t ld_scores, void *stream);

/* a8 / §8(f)1 -- evaluation ranking (src/model/KGAT/main.py:70-130, 576-605;
 * src/utils/metrics_calculator.py:84-131).
 * kgat_mask_rows_f32: scores[r, idx[e]] = value for e in [rowptr[r], rowptr[r+1])
 *   (the reference's `cf_scores[idx][train_items] = -inf`; out-of-range ids skipped).
 * kgat_topk_f32: per row the k (<= 1024, <= cols) largest scores, descending;
 *   equal scores by ascending column (torch.sort/topk leave tie order unspecified).
 *   out_idx int32 [rows, k]; out_val (nullable) float [rows, k].
 * kgat_rank_metrics_f32: from top-k columns (kmax per row) and each row's sorted,
 *   unique test items (CSR), writes out[t][m][r] for k_list[t] (host array,
 *   n_k <= 16, each <= kmax) and m = precision, recall, ndcg -- the formulas of
 *   metrics_calculator.py:17-81 (recall of a row with no test items is nan). */
int kgat_mask_rows_f32(float *scores, int64_t ld, int32_t rows, int32_t cols, const int64_t *rowptr,
                       const int32_t *idx, float value, void *stream);
int kgat_topk_f32(const float *scores, int64_t ld, int32_t rows, int32_t cols, int32_t k, int32_t *out_idx,
                  float *out_val, void *stream);
int kgat_rank_metrics_f32(const int32_t *topk_idx, int32_t rows, int32_t kmax, const int64_t *test_rowptr,
                          const int32_t *test_idx, const int32_t *k_list, int32_t n_k, float *out, void *stream);

/* a10/a11 -- NFM (src/model/NFM/model.py:73-129).  Parameters by pointer:
 * V [F, dims[0]] (row stride ld_v), wide head w_lin [F] + b_lin [1], hidden
 * layers W[l] [dims[l+1], dims[l]] / b[l], output W_out [dims[L]] (no bias).
 * dropout_p > 0: train-mode dropout after every hidden ReLU (hash mask). */
#define KGAT_NFM_MAX_LAYERS 4
typedef struct kgat_nfm {
  const float *V;
  int64_t ld_v;
  const float *w_lin;
  const float *b_lin;
  const float *W[KGAT_NFM_MAX_LAYERS];
  const float *b[KGAT_NFM_MAX_LAYERS];
  int32_t dims[KGAT_NFM_MAX_LAYERS + 1];
  int32_t n_layers;
  const float *W_out;
  float dropout_p;
  uint64_t seed;
} kgat_nfm;

/* CSR row pointers [n_rows + 1] of a row-sorted COO row array. */
int kgat_coo_rowptr(const int64_t *rows_sorted, int64_t nnz, int64_t n_rows, int64_t *rowptr, void *stream);
/* Scores y[r] for a CSR feature batch (bi-interaction pooling + MLP + heads);
 * act (nullable, kgat_nfm_act_floats) keeps what the backward needs. */
int64_t kgat_nfm_act_floats(const kgat_nfm *net, int64_t rows);
int kgat_nfm_fwd_f32(const kgat_nfm *net, const int64_t *rowptr, const int64_t *col, const float *val,
                     int64_t rows, float *act, float *y, void *stream);
/* BPR loss over rows [0, batch) = positives and [batch, 2*batch) = negatives:
 * -mean log(1e-10 + sigmoid(y_pos - y_neg)) + lam |W_out|^2 / 2; dy = dL/dy. */
int kgat_nfm_loss_f32(const kgat_nfm *net, const float *y, int32_t batch, float lam, float *loss, float *dy,
                      void *stream);
/* Backward: dV (dense, zero-initialised) and dw_lin (zero-initialised) get the
 * feature gradients (entries: erow/col/val, duplicates summed in entry order;
 * feature ids < 2^32, nnz < 2^31); dW[l], db[l], dW_out, db_lin are overwritten.
 * kgat_nfm_bwd_workspace: floats of workspace for (rows, nnz), -1 if invalid. */
int64_t kgat_nfm_bwd_workspace(const kgat_nfm *net, int64_t rows, int64_t nnz);
int kgat_nfm_bwd_f32(const kgat_nfm *net, const int64_t *erow, const int64_t *col, const float *val, int64_t nnz,
                     int64_t rows, const float *act, const float *dy, const float *grad_out, float lam, float *dV,
                     int64_t ld_dv, float *dw_lin, float *db_lin, float *const *dW, float *const *db,
                     float *dW_out, float *workspace, int64_t workspace_floats, void *stream);

/* a9 -- one dense Adam step for one tensor, torch.optim.Adam semantics
 * (model.py:404-419): m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g g;
 * p -= step_size * m / (sqrt(v)/bc2_sqrt + eps). */
int kgat_adam_f32(float *p, const float *g, float *m, float *v, int64_t n, float step_size, float beta1,
                  float beta2, float bc2_sqrt, float eps, void *stream);

/* a9 for every tensor of one optimiser step in ONE launch (up to 16 tensors):
 * per tensor the arguments of kgat_adam_f32.  Same arithmetic, bit for bit. */
#define KGAT_ADAM_MAX_TENSORS 16
typedef struct kgat_adam_tensor {
  float *p;
  const float *g;
  float *m;
  float *v;
  int64_t n;
  float step_size;
  float bc2_sqrt;
} kgat_adam_tensor;
int kgat_adam_multi_f32(const kgat_adam_tensor *tensors, int32_t count, float beta1, float beta2, float eps,
                        void *stream);
/* ... with the optimiser skip flag (see kgat_spmm_csr_masked_adam_ex_f32). */
int kgat_adam_multi_ex_f32(const kgat_adam_tensor *tensors, int32_t count, float beta1, float beta2, float eps,
                           const int32_t *skip, void *stream);
/* kgat_spmm_csr_masked_adam_ex_f32 that also steps n_extra (<= KGAT_ADAM_MAX_TENSORS) further tensors in
 * its second launch: the long rows' fix-up and kgat_adam_multi_ex_f32's step of `extra` (same beta1 /
 * beta2 / eps and skip flag, each tensor its own step size and bias correction) share one launch -- the
 * CF step's table update and the aggregator weights' Adam (model.py:404-413), bit for bit the two calls.
 * n_extra = 0: kgat_spmm_csr_masked_adam_ex_f32. */
int kgat_spmm_csr_masked_adam_multi_f32(const kgat_csr *A, const int32_t *src_map, const float *Xc, int64_t ldxc,
                                        const float *Yc_init, int64_t ldyc, const uint64_t *src_rank, float *p,
                                        float *m, float *v, int64_t ldp, int32_t d, float step_size, float beta1,
                                        float beta2, float bc2_sqrt, float eps, const int32_t *skip,
                                        float *workspace, int64_t workspace_floats, const kgat_adam_tensor *extra,
                                        int32_t n_extra, void *stream);

/* a9 for the KG step's table (model.py:414-419 after the TransR backward, whose table gradient is
 * nonzero on the <= 3B rows of the batch only): the dense Adam step over p / m / v [n_rows x d]
 * where row r's gradient is Gc[row_map[r]] (ldg floats per compact row) when row_map[r] >= 0 and
 * 0 otherwise -- the same bits as kgat_adam_f32 on the dense zero-filled gradient, which is never
 * written.  d % 4 == 0, 16-byte aligned arrays. */
int kgat_adam_rows_f32(float *p, float *m, float *v, int64_t n_rows, int32_t d, const int32_t *row_map,
                       const float *Gc, int64_t ldg, float step_size, float beta1, float beta2, float bc2_sqrt,
                       float eps, const int32_t *skip, void *stream);

/* Lazy table Adam for the KG phase (KGAT.lazy_kg_adam): the dense step moves every row each step
 * (rows outside the batch with a zero gradient); here row r records the last step applied to it
 * (last[r]) and its skipped zero-gradient steps are replayed in order -- each with its own step size,
 * bias correction and skip flag, kept in a device history of cap entries (step s at s % cap) -- when
 * it is next read or updated, or at a flush.  Every element goes through the dense step's sequence of
 * adam_elem operations: same bits.  d divides 256 (<= 256).
 * kgat_adam_lazy_catchup_f32: the listed rows (rows null: all n_rows) brought up to step t.
 * kgat_adam_lazy_rows_f32: step t (>= 1) on the listed rows with their compact gradients Gc[k]
 * (kgat_frontier_build's order; the rows' skipped steps replayed first), step t's scalars and skip flag
 * (*skip, nullable) recorded for the other rows.  A caller keeps t - min(last) < cap (flush before). */
int kgat_adam_lazy_catchup_f32(float *p, float *m, float *v, int64_t n_rows, int32_t d, const int32_t *rows,
                               int64_t n_list, int32_t *last, int32_t t, float *hist_sz, float *hist_bc,
                               int32_t *hist_skip, int32_t cap, float beta1, float beta2, float eps, void *stream);
int kgat_adam_lazy_rows_f32(float *p, float *m, float *v, int32_t d, const int32_t *rows, int64_t n_list,
                            const float *Gc, int64_t ldg, int32_t *last, int32_t t, float *hist_sz, float *hist_bc,
                            int32_t *hist_skip, int32_t cap, float step_size, float beta1, float beta2,
                            float bc2_sqrt, float eps, const int32_t *skip, void *stream);

/* The KG step captured as a HIP graph (KGAT.capture_kg_step; main.py:324-345, model.py:204-261,
 * 414-419): a graph replays the kernel arguments it was captured with, so a step's scalars live on
 * the device.  t_dev (int32 [1]) holds the optimiser's step number; the _sched variants read t = *t_dev
 * (+ t_add, below) and the step's size and
 * sqrt(1 - beta2^t) from the schedule tables sched_sz[t] / sched_bc[t] (float, > t entries, filled by
 * the host with the by-value launches' own float values: lr / (1 - beta1^t), sqrt(1 - beta2^t)).
 * Otherwise each is kgat_adam_multi_ex_f32 (every tensor at step t), kgat_adam_lazy_catchup_f32 and
 * kgat_adam_lazy_rows_f32, bit for bit. */
int kgat_adam_multi_sched_f32(const kgat_adam_tensor *tensors, int32_t count, float beta1, float beta2, float eps,
                              const int32_t *skip, const int32_t *t_dev, const float *sched_sz, const float *sched_bc,
                              int32_t t_add, int32_t *t_out, void *stream);
int kgat_adam_lazy_catchup_sched_f32(float *p, float *m, float *v, int64_t n_rows, int32_t d, const int32_t *rows,
                                     int64_t n_list, int32_t *last, const int32_t *t_dev, float *hist_sz,
                                     float *hist_bc, int32_t *hist_skip, int32_t cap, float beta1, float beta2,
                                     float eps, void *stream);
/* row_map (nullable): the batch rows' kgat_frontier_build map entries are reset to -1 by the same launch
 * (kgat_frontier_reset folded in; a skipped step resets them too).  t_add / t_out (kgat_adam_multi_sched_f32
 * and kgat_adam_lazy_rows_sched_f32): the step applied is *t_dev + t_add, and its number is written to
 * t_out (nullable) -- the captured KG update applies step *t + 1 in the lazy rows' launch, hands it on
 * through a second cell, and the relation / trans Adam writes it back to t (no separate counter launch).
 * Both write t_out before a set skip flag returns, so a skipped step advances the counter as
 * FusedAdam's step count does. */
int kgat_adam_lazy_rows_sched_f32(float *p, float *m, float *v, int32_t d, const int32_t *rows, int64_t n_list,
                                  const float *Gc, int64_t ldg, int32_t *last, float *hist_sz, float *hist_bc,
                                  int32_t *hist_skip, int32_t cap, const int32_t *t_dev, const float *sched_sz,
                                  const float *sched_bc, float beta1, float beta2, float eps, const int32_t *skip,
                                  int32_t *row_map, int32_t t_add, int32_t *t_out, void *stream);

/* dst[i] = src[idx[i]] (int32 idx) -- used to refresh transposed CSR values. */
int kgat_gather_f32(const float *src, const int32_t *idx, int64_t n, float *dst, void *stream);

/* Id validation without a host synchronisation (the reference's embedding gathers raise
 * IndexError, src/model/KGAT/model.py:188-191, 219-222, 389-391): the ids of up to
 * KGAT_IDS_MAX int64 arrays are copied, concatenated, into out; an id outside [0, bound)
 * is written as 0 (so no later kernel indexes out of range) and sets *bad to 1 (a plain
 * store: bad may be device memory or host-mapped pinned memory the caller reads after the
 * stream passes this call; the caller zeroes it). */
#define KGAT_IDS_MAX 4
typedef struct kgat_ids {
  const int64_t *ptr[KGAT_IDS_MAX];
  int64_t n[KGAT_IDS_MAX];
  int32_t count;
} kgat_ids;
int kgat_ids_check(const kgat_ids *ids, int64_t bound, int64_t *out, int32_t *bad, void *stream);
/* ... that also sets *bad_dev = 1 (device int32, nullable) -- the skip flag the optimiser kernels
 * read (kgat_adam_multi_ex_f32, kgat_spmm_csr_masked_adam_ex_f32, kgat_adam_rows_f32), so a step
 * with a bad id moves no parameter although the host learns of it later (no synchronisation);
 * the caller zeroes it after reporting the error. */
int kgat_ids_check_ex(const kgat_ids *ids, int64_t bound, int64_t *out, int32_t *bad, int32_t *bad_dev,
                      void *stream);
/* ... with one bound per array (bounds[k] for ids->ptr[k]): the KG step's heads / tails (node count) and
 * relations (relation count) checked and copied in one launch (the captured step's static input). */
int kgat_ids_check_multi(const kgat_ids *ids, const int64_t *bounds, int64_t *out, int32_t *bad, int32_t *bad_dev,
                         void *stream);

/* node_map[ids[i]] = i for i < n (ids distinct; negative ids skipped): the node -> compact row
 * map of a row list (the row-sharded backward's global batch rows, whose compact order is the
 * host's sorted unique ids).  kgat_frontier_reset(ids, n, node_map) restores -1. */
int kgat_map_build(const int32_t *ids, int64_t n, int32_t *node_map, void *stream);

/* kgat_map_build for a row list gathered from other processes (the row-sharded hop backward's
 * all-peer gather of every rank's hop rows, sharded.py _hop_layer), which nothing on this rank
 * has validated: an entry outside [-1, n_nodes) is not mapped, is overwritten with -1 (so
 * kgat_frontier_reset skips it too), and sets *bad_host (pinned host-mapped memory, may be null)
 * and *bad_dev (the optimiser kernels' skip flag, may be null).  No out-of-range access. */
int kgat_map_build_checked(int32_t *ids, int64_t n, int32_t *node_map, int64_t n_nodes, int32_t *bad_host,
                           int32_t *bad_dev, void *stream);

/* The same check without a map: ids[i] outside [-1, bound) is overwritten with -1 and sets the
 * flags (the row-sharded frontier forward's gathered row-set ids, before they place rows). */
int kgat_ids_sanitize_i32(int32_t *ids, int64_t n, int64_t bound, int32_t *bad_host, int32_t *bad_dev,
                          void *stream);

/* out[i] = a[i] < 0 ? -1 : (b ? b[a[i]] : a[i]) + offset, -1 where b[a[i]] < 0 (out may alias a
 * when b is null).  Index plumbing of the row-sharded hop backward: a batch row's compact index
 * -> its position in a hop list (b = the hop list's node map), local -> global row ids (b null,
 * offset = the shard's first row). */
int kgat_map_compose(const int32_t *a, int64_t n, const int32_t *b, int32_t offset, int32_t *out, void *stream);

/* Fill n floats with a value. */
int kgat_fill_f32(float *dst, int64_t n, float value, void *stream);

/* Row movers of the row-sharded mode (§8(e) C5): dst[i] = src[rows[i]] (rows[i] < 0
 * -> zero row); dst[rows[i]] (+)= src[i] (rows[i] < 0 skipped; rows must be
 * distinct); y += x.  d % 4 == 0, 16-byte aligned rows. */
int kgat_gather_rows_f32(const float *src, int64_t lds, const int32_t *rows, int64_t n, int32_t d, float *dst,
                         int64_t ldd, void *stream);
int kgat_scatter_rows_f32(float *dst, int64_t ldd, const int32_t *rows, int64_t n, int32_t d, const float *src,
                          int64_t lds, int32_t accumulate, void *stream);
int kgat_add_f32(float *y, const float *x, int64_t n, void *stream);

/* §8(d) synthetic CKGs at C4/C5 size, §8(f)3 graph build (host, csrc/synth.cpp).
 * Replaces, for the row-sharded configs, the reference's input-layout producer
 * (src/model/KGAT/preprocess.py:177-246, 628-634: per-relation blocks normalised
 * to A^T D^-1, summed into the attentive matrix).  Each draw is a pure function
 * of (seed, stream, index), so every rank builds only its own rows [lo, hi):
 *   kgat_synth_open         finds the first n_triples distinct triples of the seeded
 *                           draw streams (repeats dropped and redrawn),
 *                           counts the degrees (all kept triples, n_threads); n_nodes
 *                           < 2^30
 *   kgat_synth_info         info[8] = {n_nodes, n_triples, users, entities, items,
 *                           interactions, kg_triples, draws taken} (n_triples = the
 *                           kept count: smaller only when the type ranges cannot hold
 *                           that many distinct triples)
 *   kgat_synth_row_offsets  [n_nodes + 1] prefix sums of each row's pre-coalesce
 *                           entries (the balance weights of the row shards)
 *   kgat_synth_triples      raw triples by index: rel = -1 -> (user a, item b),
 *                           else KG (head a, rel, tail b), entity ids
 *   kgat_synth_shard_build  coalesced CSR of rows [lo, hi) (global column ids), kept
 *                           in the handle; *nnz = its entry count
 *   kgat_synth_shard_copy   copies it to rowptr [hi-lo+1] (0-based), col, val [nnz]
 *                           (host memory) and releases the handle's copy.
 * Host-only; no HIP call.  Status codes as everywhere else. */
typedef struct kgat_synth kgat_synth;
int kgat_synth_open(int64_t n_nodes, int64_t n_triples, uint64_t seed, double zipf_s, int n_threads,
                    kgat_synth **out);
void kgat_synth_close(kgat_synth *g);
int kgat_synth_info(const kgat_synth *g, int64_t *info);
int kgat_synth_row_offsets(const kgat_synth *g, int64_t *offsets);
int kgat_synth_triples(const kgat_synth *g, const int64_t *idx, int64_t count, int64_t *a, int32_t *rel,
                       int64_t *b);
int kgat_synth_shard_build(kgat_synth *g, int64_t lo, int64_t hi, int64_t *nnz);
/* transpose != 0: rows [lo, hi) of A^T (the row-sharded backward's AT_loc, sharded.RowShard) --
 * bit for bit the transpose of the layout's A restricted to those rows. */
int kgat_synth_shard_build_ex(kgat_synth *g, int64_t lo, int64_t hi, int32_t transpose, int64_t *nnz);
int kgat_synth_shard_copy(kgat_synth *g, int64_t *rowptr, int32_t *col, float *val);

/* (e) Multi-GPU transport: an RCCL communicator over xGMI behind
 * an opaque handle, one process per GPU.  No reference counterpart -- the
 * reference is single-device (src/model/KGAT/main.py:239); these are the
 * collectives of the data-parallel replicas (replicas.py: table-gradient
 * reduce-scatter / all-gather, hop-set all-gathers, the small-gradient
 * all-reduce) and of the row-sharded propagation ring (sharded.py).  RCCL is
 * bound at run time: kgat_comm_load(path) picks the library (NULL:
 * "librccl.so.1"; a host that already carries an RCCL passes its path so the
 * process holds one instance); the other calls load the default on first use.
 * Every collective is stream-ordered on `stream`.  Errors: KGAT_ERR_COMM_BASE +
 * ncclResult_t (kgat_comm_error_string), KGAT_ERR_COMM_UNAVAILABLE. */
#define KGAT_COMM_ID_BYTES 128
typedef struct kgat_comm kgat_comm;
int kgat_comm_load(const char *rccl_path);
const char *kgat_comm_error_string(int status);
/* rank 0 makes the id and shares it out of band (e.g. a TCP store) */
int kgat_comm_unique_id(uint8_t *id);
int kgat_comm_init(int32_t rank, int32_t world, const uint8_t *id, int32_t device, kgat_comm **out);
int kgat_comm_destroy(kgat_comm *comm);
int kgat_comm_rank(const kgat_comm *comm, int32_t *rank, int32_t *world);
/* recv = sum over ranks of send (count floats; send == recv in place) */
int kgat_comm_allreduce_sum_f32(kgat_comm *comm, const float *send, float *recv, int64_t count, void *stream);
/* recv[r * bytes_per_rank ..] = rank r's send (rank order; send may alias recv + rank * bytes_per_rank) */
int kgat_comm_allgather_rows(kgat_comm *comm, const void *send, void *recv, int64_t bytes_per_rank, void *stream);
/* recv (count_per_rank floats) = sum over ranks of send[rank * count_per_rank ..] (row blocks) */
int kgat_comm_reduce_scatter_rows_f32(kgat_comm *comm, const float *send, float *recv, int64_t count_per_rank,
                                      void *stream);
/* the propagation ring's step: send -> rank + 1, rank - 1 -> recv (bytes each) */
int kgat_comm_ring_exchange(kgat_comm *comm, const void *send, void *recv, int64_t bytes, void *stream);
/* Uneven all-gather over every peer link at once (the row-sharded layer gather, sharded.py): rank
 * r's block is recv[offsets[r], offsets[r+1]) (byte offsets, world + 1 of them, the same on every
 * rank); this rank's block comes from send (which may alias recv + offsets[rank]).  One send and
 * one receive per peer in a single RCCL group -- on a fully connected xGMI node every peer pair
 * has its own link, so all seven links carry rows concurrently (no ring hop). */
int kgat_comm_allgatherv(kgat_comm *comm, const void *send, void *recv, const int64_t *offsets, void *stream);
/* The same gather with every rank's block placed anywhere: rank r's nbytes[r] bytes land at
 * recv + dst_off[r] (world entries each, the same on every rank; blocks must not overlap).  The
 * row-sharded forward posts each finished row block of a layer's output with it (rank r's block b =
 * rows [lo_r + a_rb, lo_r + a_r(b+1)) of the next layer's gathered input), so the next layer's wire
 * time runs under this layer's remaining blocks.  World <= KGAT_COMM_MAX_WORLD. */
#define KGAT_COMM_MAX_WORLD 64
int kgat_comm_gather_at(kgat_comm *comm, const void *send, void *recv, const int64_t *dst_off, const int64_t *nbytes,
                        void *stream);
/* All-to-all with per-peer sizes: send[send_off[p], send_off[p+1]) goes to rank p, rank p's block
 * lands in recv[recv_off[p], recv_off[p+1]) (byte offsets, world + 1 each); the own block is
 * copied on the stream.  The row-sharded attention refresh moves A's refreshed values to the
 * owners of A^T's rows with it. */
int kgat_comm_alltoallv(kgat_comm *comm, const void *send, const int64_t *send_off, void *recv,
                        const int64_t *recv_off, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* KGAT_HIP_H */
