/*
 * gta.h -- C ABI of libgta, the MI355X (gfx950) execution backend for GTA's
 * message-passing ISA.
 *
 * The reference has no native code: its "execution" of an instruction stream
 * is the Python cycle model `simulate(tile_size_list, dataset, network, layer,
 * isReorder, isSinput) -> (cycles, rw)` (reference code/simulator.py:370-502),
 * fed by the stream that `interpret()` writes (code/interpreter.py:805-849).
 * Every entry point below executes, on real tensors, one ISA op or one fused
 * pattern of that stream; the Python executor
 * (gta_graph_tensor_acclelrator_for_general_gnn_amd/executor.py) walks the
 * stream block by block and calls them.  Each function cites the reference
 * construct whose semantics it executes.
 *
 * Conventions
 *  - Plain pointers and sizes only; all pointers are DEVICE pointers owned by
 *    the caller.  The library allocates nothing; plan/workspace sizes are
 *    queried with the *_bytes functions.
 *  - Graph = CSR sorted by DESTINATION row ("R" direction, the reference's
 *    row tile axis, code/preprocessing.py:26-38): int64 indptr[n_rows+1],
 *    int32 indices[nnz] = SOURCE column of each edge ("C" direction).
 *    Edge e of row i is the e-th entry of the CSR; edge tensors are [nnz, F]
 *    in CSR order.
 *  - Dense tensors are row-major with a leading dimension (elements).
 *  - Every call is asynchronous and stream-ordered on `stream` (a hipStream_t
 *    passed as void*; NULL = the default stream).  No host globals besides the
 *    thread-local error string: calls are reentrant per stream.
 *  - Return 0 on success, <0 on error; gta_last_error() gives the message of
 *    the calling thread's last failure.
 */
#ifndef GTA_H_
#define GTA_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GTA_ABI_VERSION 14 /* 2: blocked plans of bounded items (nnz, item_edges); 3: per-thread tuning
                              hooks; 4: knob sets attached to streams (gta_tuning_*); 5: every UPDATE
                              on hand-written kernels (no vendor library), gta_update_mm_t_splits,
                              the blocked workspace is the slab rows alone and required, bf16
                              rows in gta_aggregate (x_dtype) and gta_apply_node (a_dtype);
                              6: gta_gat_aggregate_blocked's sf_out (an SF applied to y); 7:
                              gta_aggregate_self (the aggregate with a scaled self term); 8:
                              gta_update_mm_t_splits takes the stream (its attached knob set); 9:
                              gta_update_mlp (two chained node GEMMs in one pass); 10: bf16 y of
                              gta_aggregate_self, bf16 x of gta_update_mlp; 11: gta_gather_add takes the ISA
                              DIRECTION (dir R / C) and the CSC view of gta_csc_build; 12:
                              gta_build_id, gta_synth_alpha and gta_row_ids (scan-free setup); 13: gta_apply_edge_flat;
                              14: gta_aggregate_expr */

/* status codes */
enum { GTA_OK = 0, GTA_ERR_ARG = -1, GTA_ERR_HIP = -2, GTA_ERR_UNSUPPORTED = -3 };

/* dtypes; GTA_F32_BF16 (update_mm only): fp32 x rounded to bf16 (RNE) as it is
 * staged into LDS, bf16 W -- no separate cast pass over x */
enum { GTA_F32 = 0, GTA_BF16 = 1, GTA_F32_BF16 = 2 };

/* Scatter direction (reference ISA `scatter` DIRECTION dst/src,
 * template/ISA_defination.yaml:33-44; op ORDER R/C in the op YAML). */
enum { GTA_DIR_R = 0, /* edge takes its DESTINATION row's feature */
       GTA_DIR_C = 1  /* edge takes its SOURCE column's feature   */ };

/* How an edge-indexed operand addresses its rows. */
enum { GTA_IDX_EDGE = 0, /* row e of an edge tensor [nnz, F]            */
       GTA_IDX_SRC = 1,  /* row indices[e] of a node tensor (scatter C) */
       GTA_IDX_DST = 2   /* row i (edge's destination) (scatter R)      */ };

/* Binary element-wise compute types of applyedge/applynode (COMP_TYPE in the
 * op YAML, vTCAD/GraphOP/genGraphOP.py:4-25).  DIV is the "/" of
 * template/GAT_op.png op 9 (typed MUL in the YAML). */
enum { GTA_BIN_NONE = 0, GTA_BIN_ADD = 1, GTA_BIN_MUL = 2, GTA_BIN_DIV = 3, GTA_BIN_SUB = 4 };

/* Special functions (COMP_TYPE "SF", unit SF_ALU, code/interpreter.py:7).
 * The reference never fixes which function an SF is; these are the build's
 * choices, applied as a post-op of the producing kernel. */
enum { GTA_SF_NONE = 0, GTA_SF_RELU = 1, GTA_SF_EXP_LEAKY_RELU = 2 /* exp(leaky_relu(x,0.2)) */,
       GTA_SF_ELU = 3, GTA_SF_EXP = 4, GTA_SF_LEAKY_RELU = 5, GTA_SF_SIGMOID = 6,
       GTA_SF_TANH = 7, GTA_SF_RECIP = 8 };

int gta_abi_version(void);
const char* gta_last_error(void);
/* ABI 12: the first 16 hex digits of sha256(csrc/gta_kernels.hip || include/gta.h) the library
 * was compiled from ("unversioned" when built without _build.py).  The Python binding refuses a
 * library whose id differs from the sources beside it. */
const char* gta_build_id(void);

/* Tuning hooks (benchmarks and kernel-form tests): named knobs that pick between kernel forms
 * the defaults reach on some shape, or split a launch for per-kernel timing.  They are per calling THREAD -- a knob set on one thread never
 * changes another thread's concurrent calls -- and every entry point reads its own thread's
 * values, so the library keeps no process-wide mutable state.  Unknown key: GTA_ERR_ARG. */
int gta_debug_set(const char* key, int64_t value);
int gta_debug_get(const char* key, int64_t* value);

/* Knob sets scoped to a STREAM (ABI 4): a handle holds a full set of knobs (the defaults until
 * set); gta_tuning_attach(stream, h) copies h's values onto the stream, and from then on every
 * call made on that stream -- from any thread -- reads that copy, taken at the call's entry,
 * instead of the calling thread's knobs.  h may be changed or destroyed after attaching (attach
 * again to apply changes); h == NULL detaches.  Streams without an attached set use the calling
 * thread's knobs (gta_debug_set), so concurrent calls on different streams never see each
 * other's settings.  The set is keyed by the raw hipStream_t value: detach before destroying the
 * stream (a stream created later may reuse the handle and would inherit the set), and a set
 * attached to the null stream (NULL) governs every call made on the default stream. */
typedef struct gta_tuning gta_tuning;
gta_tuning* gta_tuning_create(void);
void gta_tuning_destroy(gta_tuning* h);
int gta_tuning_set(gta_tuning* h, const char* key, int64_t value);
int gta_tuning_get(const gta_tuning* h, const char* key, int64_t* value);
int gta_tuning_attach(void* stream, const gta_tuning* h);

/* ---- K1 SCATTER (node -> edge copy) -------------------------------------
 * out[e, :] = x[dir==R ? dst(e) : src(e), :]          (bit-exact copy)
 * Reference: ISA `scatter` template/ISA_defination.yaml:33-44; lowered as
 * LOAD_N + FETCH + STORE_E, code/interpreter.py:49-53, 62-68, 367-372. */
int gta_scatter(int dir, const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t nnz,
                const void* x, int64_t ldx, int64_t F, int dtype, void* out, int64_t ldo, void* stream);

/* ---- K6/K7/K2 AGGREGATE (fused applyedge MUL -> gather ADD) -------------
 *   y[i, c] (+)= row_scale[i] * sum_{e in row i} w(e, c) * x[idx(e), c]
 * x_mode = GTA_IDX_SRC: the fused scatter-C FETCH (weighted/unweighted SpMM,
 *          COMP_MUL_COMP_ADD of block [3,11,12] in GAT, [0,1,2] in GCN/SAGE/GIN);
 *          GTA_IDX_EDGE: a plain gather ADD of an edge tensor (K2);
 *          GTA_IDX_DST : the fused scatter-R FETCH.
 * w: NULL (unweighted, pattern [scatter,gather] (NONE,ADD)) or [nnz, ldw]
 *    with `heads` columns: column c uses w[e, c / (F/heads)]  (heads | F;
 *    heads == F is a full-width edge tensor, heads == 1 a scalar edge weight).
 * row_scale: NULL or float[n_rows] (e.g. 1/deg for SAGE-mean).
 * plan: NULL (one wavefront per row) or a plan built by
 *       gta_aggregate_plan_build with the same graph and plan_chunk; rows
 *       longer than plan_chunk are split over several wavefronts whose
 *       partials are summed in a fixed order (deterministic; no atomics).
 * x_dtype: GTA_F32, or GTA_BF16 for x_mode SRC / DST with w NULL or head weights
 *          (rows widened exactly to fp32, sums in fp32: the 2-byte gathers of BASELINE.md's
 *          GIN byte model).
 * workspace: >= gta_aggregate_workspace_bytes(...) when plan != NULL.
 * Reference: hardware_info.yaml Inst_fused [applyedge,gather] [MUL,ADD]
 * ("FinalVersion For Paper/hardware_info.yaml":35-38), inst_fusion_x2
 * code/interpreter.py:575-636, fuse_fetch :764-802; gather ISA
 * template/ISA_defination.yaml:46-61. */
int gta_aggregate(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t nnz,
                  int x_mode, const void* x, int64_t ldx, int64_t F, int x_dtype,
                  const float* w, int64_t ldw, int64_t heads,
                  const float* row_scale, float* y, int64_t ldy, int accumulate,
                  const void* plan, int64_t plan_chunk, void* workspace, void* stream);

/* ABI 14: the aggregate of an apply_edge expression -- a gather R whose edge value is a tree of
 * K3 ops over up to four operand rows, with no [E, F] edge tensor written for any of them:
 *   shape 1: t = sf0(L0 bin0 L1)                 (bins[0] GTA_BIN_NONE: t = sf0(L0), one operand)
 *   shape 2: u = sf0(L0 bin0 L1); t = sf1(swap ? L2 bin1 u : u bin1 L2)
 *   shape 3: u = sf0(L0 bin0 L1); v = sf1(L2 bin1 L3); t = sf2(u bin2 v)
 *   y[i, :] = sum_{e in row i} t(e, :)
 * Operand l is operands[l] (fp32, F columns, row stride lds[l]) read per modes[l]: GTA_IDX_EDGE
 * (row e; lds 0 = one row broadcast to every edge), GTA_IDX_SRC (row indices[e]), GTA_IDX_DST
 * (row i).  Every step is the gta_apply_edge arithmetic with the intermediate rounded to fp32 as its
 * stored output would be, and the sum runs in gta_aggregate(x_mode EDGE)'s order with the same
 * plan: bitwise equal to the apply_edge ops followed by that aggregate of their [E, F] output.
 * GTA_ERR_UNSUPPORTED when an operand's alignment or stride does not admit the vector width that
 * aggregate would use for F (then run the ops unfused).  operands / modes / lds / bins / sfs are
 * host arrays read during the call.  DGN ops 2-8 (the MM of op 3 pushed to the node rows) and PNA
 * ops 5-8 of the genGraphOP op graphs (restated in frontend.py). */
int gta_aggregate_expr(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t nnz, int shape,
                       const float* const* operands, const int* modes, const int64_t* lds, const int* bins,
                       const int* sfs, int swap, int64_t F, float* y, int64_t ldy, const void* plan,
                       int64_t plan_chunk, void* workspace, void* stream);

/* ABI 7: the aggregate with a self term, y[i, :] = self_scale[0] * x_self[i, :] + row_scale[i] *
 * sum_{e in row i} w(e) x[idx(e), :] (no accumulate).  x_self has x's dtype and F columns (ld_self
 * >= F); self_scale is a DEVICE pointer to one float (NULL = 1), so a captured graph follows it.
 * The self term is formed as an applynode MUL by a broadcast scalar forms it, each product rounded
 * (no fma contraction): with row_scale NULL, bitwise equal to gta_apply_node(MUL, x_self, s) into y
 * then gta_aggregate accumulating into y; with row_scale, the scaled sum is rounded before the add
 * (the unfused scaled aggregate, then ADD).  GIN ops 3-4
 * (genGraphOP.py:99-103): agg + (1 + eps) x with no [N, F] intermediate.
 * y_dtype (ABI 10): GTA_F32, or GTA_BF16 -- y holds the RNE bf16 rounding of the fp32 value (ldy in
 * bf16 elements), for a consumer that rounds its input to bf16 anyway (gta_update_mlp: GIN's MLP
 * after ops 3-4), so half the bytes are written and read and the value it sees is unchanged. */
int gta_aggregate_self(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t nnz, int x_mode,
                       const void* x, int64_t ldx, int64_t F, int x_dtype, const float* w, int64_t ldw, int64_t heads,
                       const float* row_scale, const void* x_self, int64_t ld_self, const float* self_scale, void* y,
                       int64_t ldy, int y_dtype, const void* plan, int64_t plan_chunk, void* workspace, void* stream);

/* plan/workspace sizing: chunk must be a positive multiple of 64 */
int64_t gta_aggregate_plan_bytes(int64_t n_rows, int64_t nnz, int64_t chunk);
int gta_aggregate_plan_build(const int64_t* indptr, int64_t n_rows, int64_t nnz, int64_t chunk,
                             void* plan, int64_t plan_bytes, void* stream);
int64_t gta_aggregate_workspace_bytes(int64_t n_rows, int64_t nnz, int64_t chunk, int64_t F);

/* ---- K6 column-blocked form (L2-resident source slices) -----------------
 * Same y as gta_aggregate (x_mode SRC, w NULL or heads), computed over B source-column
 * blocks [b*ceil(n_cols/B), (b+1)*ceil(n_cols/B)): the work items of one block run
 * together, so the waves in flight gather from one X slice that stays resident in
 * each XCD's 4 MB L2 -- the reference's own
 * T-row x column tiling (code/preprocessing.py:26-38, interpreter TC) with the
 * column axis outermost.  Needs each CSR row's columns sorted (the plan build
 * flags unsorted rows in plan header word 3) and F = 64*VW (64/128/256) with
 * (F/heads)/VW in {4, 8, 16}.  Deterministic (fixed block order, no atomics);
 * row_scale is applied per block.  1 <= blocks <= 63.
 * The plan cuts every (block, row) segment into ceil(len / item_edges) work
 * items of near-equal length (the reference's tile split of a long row,
 * Tile_Times per row tile, code/interpreter.py:244-259): a heavy row's gathers
 * then spread over several waves instead of one long chain at the launch tail.
 * row_edges > 0 merges column blocks for light rows: a row of deg edges uses
 * blocks of m fine blocks (m the power of two >= row_edges * blocks / deg, at
 * most blocks), so its items still hold ~row_edges edges; 0 = every row uses
 * all blocks.  Only the plan build takes it (any value keeps y within fp32
 * rounding; the sum order per row is fixed by the plan).
 * plan, workspace and launch must use the same (nnz, blocks, item_edges). */
int64_t gta_aggregate_blocked_plan_bytes(int64_t n_rows, int64_t nnz, int64_t blocks, int64_t item_edges);
int gta_aggregate_blocked_plan_build(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t n_cols,
                                     int64_t nnz, int64_t blocks, int64_t item_edges, int64_t row_edges,
                                     void* plan, int64_t plan_bytes, void* stream);
/* workspace >= gta_aggregate_blocked_workspace_bytes (may be NULL only when nnz == 0):
 * one launch over the plan's items in block-major order, item k writing partial row
 * k, then an ordered reduce summing each row's items in (block, part) order. */
int64_t gta_aggregate_blocked_workspace_bytes(int64_t n_rows, int64_t nnz, int64_t blocks, int64_t F,
                                              int64_t item_edges);
int gta_aggregate_blocked(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t n_cols, int64_t nnz,
                          const float* x, int64_t ldx, int64_t F, const float* w, int64_t ldw, int64_t heads,
                          const float* row_scale, float* y, int64_t ldy, int accumulate, const void* plan,
                          int64_t blocks, int64_t item_edges, void* workspace, void* stream);

/* ---- K6' fused GAT attention aggregate (GAT ops 6-12 without the final SF) ----
 * v(e, h) = sf( a_dst[dst(e), h] + b_src[src(e), h] )
 * normalize: y[i, c] = sum_e v(e, h(c)) x[src(e), c] / sum_e v(e, h(c))   (0 for rows w/o edges)
 *            = the GAT-original chain alpha = v / sum (ops 6-10), alpha * x (op 11), gather (op 12)
 * else:      y[i, c] = sum_e v(e, h(c)) x[src(e), c]     (GAT-trans numerator, op 10)
 * sums[i, h] = sum_e v(e, h) if sums != NULL (GAT-trans denominator, op 9).  h(c) = c / (F/heads).
 * sf_out (ABI 6): GTA_SF_NONE, or an SF applied to every y element as it is written -- the
 * applynode SF that follows the aggregate (GAT op 13, genGraphOP.py:64); rows without edges get
 * sf_out(0).  Same function as gta_apply_node's SF: bitwise equal to y then gta_apply_node. 
 * Column-blocked like gta_aggregate_blocked (same plan; rows' columns sorted): the score
 * table b is gathered beside x from the same L2-resident slice and no [E, heads] tensor is
 * ever written.  workspace >= gta_gat_aggregate_blocked_workspace_bytes.  F in {64, 128,
 * 256}, x rows 16-B aligned, (F/heads) a multiple of F/16.
 * Reference: GAT op graph vTCAD/GraphOP/genGraphOP.py:51-64; template/GAT_op.png. */
int64_t gta_gat_aggregate_blocked_workspace_bytes(int64_t n_rows, int64_t nnz, int64_t blocks, int64_t F,
                                                  int64_t heads, int64_t item_edges);
int gta_gat_aggregate_blocked(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t n_cols,
                              int64_t nnz, const float* x, int64_t ldx, int64_t F, const float* a_dst, int64_t lda,
                              const float* b_src, int64_t ldb, int64_t heads, int sf, int normalize, int sf_out,
                              float* y, int64_t ldy, float* sums, const void* plan, int64_t blocks, int64_t item_edges,
                              void* workspace, void* stream);

/* ---- CSC view of the CSR (ABI 11) -----------------------------------------
 * The edges ordered by SOURCE column, for the ISA gather / scatter with DIRECTION src
 * ("column-wise", template/ISA_defination.yaml:35, :48; ORDER C in the op YAML, lowered by
 * code/interpreter.py:55-129): colptr int64 [n_cols+1] (column j's edges are positions
 * colptr[j] .. colptr[j+1]-1), perm int32 [nnz] = the CSR edge id at each position, and
 * optionally rows int32 [nnz] = that edge's destination row (NULL: not written).  Stable:
 * within a column, edges keep their CSR order (increasing destination row), so the result is a
 * pure function of the CSR and every consumer's sum order is fixed.  A device LSD radix sort
 * (8-bit digits, ceil(log2(n_cols)/8) passes, no order decided by atomics); built once per graph.
 * indices must lie in [0, n_cols) (colptr[n_cols] == nnz then); nnz < 2^31.
 * workspace >= gta_csc_workspace_bytes(n_cols, nnz). */
int64_t gta_csc_workspace_bytes(int64_t n_cols, int64_t nnz);
int gta_csc_build(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t n_cols, int64_t nnz,
                  int64_t* colptr, int32_t* perm, int32_t* rows, void* workspace, int64_t workspace_bytes,
                  void* stream);

/* ---- K2 GATHER ADD (edge -> node), both ISA directions (ABI 11) -----------
 * dir GTA_DIR_R: y[i, :] (+)= sum_{e in row i} xe[e, :]          (to the destination, y [n_rows])
 *                == gta_aggregate(x_mode=EDGE, w=NULL); colptr / perm unused (may be NULL).
 * dir GTA_DIR_C: y[j, :] (+)= sum_{e : src(e) = j} xe[e, :]      (to the source, y [n_cols])
 *                summed in CSC order (colptr / perm of gta_csc_build): deterministic, no atomics.
 * xe is an edge tensor [nnz, F] in CSR order.
 * Reference: gather ISA DIRECTION dst/src template/ISA_defination.yaml:46-61; LOAD_E + Virtual
 * LOAD_N + COMP_ADD + STORE_N, code/interpreter.py:329-334, 373-375; tile counts per ORDER,
 * code/interpreter.py:55-129 (STORE_N of ORDER C: TR*TC x SC). */
int gta_gather_add(int dir, const int64_t* indptr, int64_t n_rows, int64_t nnz, const int64_t* colptr,
                   const int32_t* perm, int64_t n_cols, const float* xe, int64_t ldxe, int64_t F, float* y,
                   int64_t ldy, int accumulate, void* stream);

/* ---- K3' fused GAT edge-softmax (ops 6-10 of the GAT op graph) ------------
 * v(e, h)     = sf( a_dst[dst(e), h] + b_src[src(e), h] )       (ops 6 ADD, 7 SF)
 * sums[i, h]  = sum_{e in row i} v(e, h)                        (op 8 gather ADD)
 * out[e, h]   = v(e, h) / sums[dst(e), h]   if normalize        (ops 10 scatter R, 9 "/")
 *             = v(e, h)                      otherwise (GAT-trans: ops 6, 8, 9)
 * heads in {1,2,4,...,64}; out [E, heads] and sums [N, heads] contiguous; sums
 * may be NULL.  Zero in-degree rows get sums 0 and no edges.
 * Reference: GAT op graph vTCAD/GraphOP/genGraphOP.py:51-60 (ops 4-10),
 * template/GAT_op.png (alpha = exp / sum exp); SF unit code/interpreter.py:7. */
int gta_edge_softmax(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t nnz,
                     const float* a_dst, int64_t lda, const float* b_src, int64_t ldb, int64_t heads, int sf,
                     int normalize, float* out, float* sums, void* stream);

/* ---- K3 APPLYEDGE element-wise -----------------------------------------
 * out[e, c] = sf( a[ia(e), c_a] (bin) b[ib(e), c_b] )   for c < max(Fa, Fb)
 * ia/ib per GTA_IDX_*; the narrower operand is broadcast in contiguous
 * groups (head broadcast: c_b = c / (Fa/Fb)).  b may be NULL (bin ignored).
 * ldb == 0 broadcasts one row of b to every edge.
 * Reference: applyedge ops of vTCAD/GraphOP/genGraphOP.py:36, 55-60, 113-118. */
int gta_apply_edge(int bin, int sf, const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t nnz,
                   const float* a, int a_mode, int64_t lda, int64_t Fa,
                   const float* b, int b_mode, int64_t ldb, int64_t Fb,
                   float* out, int64_t ldo, void* stream);
/* ABI 13: the same op edge-parallel -- a wave takes 32 consecutive edges whatever their rows --
 * for outputs of exactly 64, 128 or 256 columns (rows aligned to 4 / 8 / 16 B).  edge_rows =
 * the destination row of each edge (int32 [nnz]; needed when an operand is GTA_IDX_DST),
 * indices = the CSR source ids (needed for GTA_IDX_SRC).  Bitwise equal to gta_apply_edge;
 * GTA_ERR_UNSUPPORTED for other widths. */
int gta_apply_edge_flat(int bin, int sf, const int32_t* edge_rows, const int32_t* indices, int64_t nnz, const float* a,
                        int a_mode, int64_t lda, int64_t Fa, const float* b, int b_mode, int64_t ldb, int64_t Fb,
                        float* out, int64_t ldo, void* stream);

/* ---- K5 APPLYNODE element-wise -----------------------------------------
 * out[i, c] = sf( a[i, c_a] (bin) b[i, c_b] ), same broadcast rules, ldb == 0
 * broadcasts one row (e.g. the (1+eps) scalar of GIN op 3).  a_dtype GTA_F32 or GTA_BF16
 * (a widened exactly); b and out fp32.
 * Reference: applynode ops genGraphOP.py:62, 94-95, 103-108. */
int gta_apply_node(int bin, int sf, int64_t n, const void* a, int64_t lda, int64_t Fa, int a_dtype,
                   const float* b, int64_t ldb, int64_t Fb, float* out, int64_t ldo, void* stream);

/* ---- K4 UPDATE / MVM on MFMA (applynode MM, applyedge MM) -------------
 * out[m, :] = sf( x[r(m), :] . W )   x: [*, K] (dtype), W: [K, N] row-major
 * (dtype; GTA_F32_BF16 = fp32 x, bf16 W), out: [M, N] fp32.  row_idx NULL => r(m) = m, else r(m) =
 * row_idx[m] (the fused [scatter, applyedge] (NONE,MM) gather-GEMM).
 * fp32 runs on v_mfma_f32_16x16x4_f32 (exact f32), bf16 on
 * v_mfma_f32_16x16x32_bf16 with fp32 accumulation.
 * Reference: applynode ISA `j,ij->i` template/ISA_defination.yaml:1-31;
 * LOAD_W + COMP_MM code/interpreter.py:335-343. */
int gta_update_mm(const void* x, int64_t ldx, const int32_t* row_idx, int64_t M, int64_t K,
                  const void* w, int64_t ldw, int64_t N, int dtype, int sf,
                  float* out, int64_t ldo, void* stream);

/* Same UPDATE with W given TRANSPOSED: wt [N, K] row-major (leading dimension
 * ldwt >= K), dtype as above.  Row-streaming kernels: a block owns up to 128 of the N
 * columns and walks row groups, so x is read once.  fp32 with N > 32, K >= 32 and 16-B
 * aligned wt rows (ldwt % 4 == 0) runs k_mm_ring: x and wt go global -> LDS by DMA through
 * a ring of 16-k stages, 3 deep for persistent blocks over many row groups, 4 at two blocks
 * per CU, 8 when every CU runs at most one block (x rows need only 4-B alignment);
 * otherwise k_mm_rows (x fragments straight to registers, wt staged per K chunk).  Both
 * contract k in the same order: bitwise equal to each other, fp32 rounding away from
 * gta_update_mm.  Every form is a hand-written kernel of this library (no vendor GEMM): the
 * result depends only on the shape and the operands, identical in every process. */
int gta_update_mm_t(const void* x, int64_t ldx, const int32_t* row_idx, int64_t M, int64_t K, const void* wt,
                    int64_t ldwt, int64_t N, int dtype, int sf, float* out, int64_t ldo, void* stream);

/* Split-K form of gta_update_mm_t for few rows (M small against the chip): the K axis is cut
 * into slices of ceil(K / splits) rounded up to 16 (every kernel form alike); each slice's
 * partial [M, N] goes to the workspace (>= gta_update_mm_t_split_workspace_bytes = splits x M x N
 * floats) and a second kernel adds the slices in order and applies sf.  Deterministic; the
 * contraction order differs from gta_update_mm_t (fp32 rounding only).  fp32 with N > 32
 * (N % 4 == 0, 16-B aligned wt rows) runs every (64-row group, slice) as one k_mm_ring block
 * with a 4-deep ring (three blocks per CU), else k_mm_rows per slice.
 * gta_update_mm_t_splits gives the slice count the library would pick for a shape on `stream`
 * (1 = no split: call gta_update_mm_t): about one (group, slice) block per CU for fp32, two for
 * bf16, slices of >= 64 k, only for K >= 256 and fewer than 128 (group, column-block) units; the
 * tuning knob mm_split overrides it -- the stream's attached knob set, else the calling thread's,
 * as for every call on a stream.  Same reference as gta_update_mm. */
int64_t gta_update_mm_t_splits(int64_t M, int64_t K, int64_t N, int dtype, void* stream);
int64_t gta_update_mm_t_split_workspace_bytes(int64_t M, int64_t K, int64_t N, int64_t splits);

/* Two chained applynode MMs with their SFs in one pass (GIN's MLP, vTCAD/GraphOP/genGraphOP.py:103-108:
 * MM -> SF -> MM -> SF; replaces two gta_update_mm_t calls and the [M, N1] intermediate they pass
 * through HBM): out = sf2(bf16(sf1(x W1)) W2).  x fp32 [M, K1] (rounded to bf16, RNE, as
 * GTA_F32_BF16 rounds it; rows 16-B aligned, K1 % 4 == 0), w1t = W1^T bf16 [N1][ldw1], w2t = W2^T bf16
 * [N2][ldw2]; K1, N1, N2 <= 128; dtype GTA_F32_BF16, or (ABI 10) GTA_BF16 for a bf16 x (ldx % 8 == 0,
 * 16-B aligned rows): then x is used as it is, and a bf16 x equal to the RNE rounding of an fp32 x
 * gives bitwise the fp32 call's result.  Other dtypes: GTA_ERR_UNSUPPORTED.  The intermediate is rounded to bf16 (RNE) exactly as the second
 * unfused GEMM's staging rounds its fp32 input, and both products run the unfused kernels' k order:
 * bitwise equal to gta_update_mm_t(x, W1, sf1) followed by gta_update_mm_t(z, W2, sf2).
 * Reference: the two COMP_MM of interpreter.py's lowering (code/interpreter.py:335-343). */
int gta_update_mlp(const void* x, int64_t ldx, int64_t M, int64_t K1, const void* w1t, int64_t ldw1, int64_t N1,
                   int sf1, const void* w2t, int64_t ldw2, int64_t N2, int sf2, int dtype, float* out, int64_t ldo,
                   void* stream);
int gta_update_mm_t_split(const void* x, int64_t ldx, const int32_t* row_idx, int64_t M, int64_t K, const void* wt,
                          int64_t ldwt, int64_t N, int dtype, int sf, float* out, int64_t ldo, int64_t splits,
                          void* workspace, int64_t workspace_bytes, void* stream);

/* ---- f2 TILE-NNZ metadata ----------------------------------------------
 * counts[t, j] = #{ distinct (dst, j) : dst in [t*T, (t+1)*T), an edge dst <- j, dst != j }
 * for t < ceil(n_rows/T), j < n_cols (int32 [ceil(n_rows/T), n_cols]).
 * A repeated column counts once when it repeats the previous entry of its row, so a CSR
 * with sorted rows (duplicates adjacent) gives exactly the dense count_nonzero of the
 * reference; the caller zeroes counts first.
 * Reference: calculate_sparsity code/preprocessing.py:12-40 (dense
 * count_nonzero per T x 1 block after removing self loops). */
int gta_tile_nnz(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t n_cols,
                 int64_t T, int32_t* counts, void* stream);

/* ---- synthetic-workload setup (ABI 12) -----------------------------------
 * Inputs of the bench's metric workload, built with one wave per row and no
 * dependency between workgroups (no device-wide scan or sort), so shards build the same way
 * however many processes share a GPU.
 * gta_synth_alpha: GAT alpha of rows [0, n_rows) of a CSR (indptr local, starting at 0) whose edge
 * e has generation id gen[e]: out[e, h] = ex[e, h] / (float)s[row, h] with
 * ex = expf(N(0,1) logit keyed by gen[e] * heads + h) and s = the row's fp64 sum of ex in edge
 * order -- the per-head softmax over in-edges of GAT ops 6-10 (vTCAD/GraphOP/genGraphOP.py:55-59).
 * The logit is the counter hash of the Python generator (graph.hash_normal, stream logit_stream).
 * heads must divide 64.
 * gta_row_ids: out[e] = the row of edge e (int64 [nnz]). */
int gta_synth_alpha(const int64_t* indptr, const int64_t* gen, int64_t n_rows, int64_t nnz, int heads, int64_t seed,
                    int64_t logit_stream, float* out, void* stream);
int gta_row_ids(const int64_t* indptr, int64_t n_rows, int64_t nnz, int64_t* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GTA_H_ */
