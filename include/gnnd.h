/*
 * gnnd.h — C ABI of libgnnd.so, the MI355X-native (gfx950) GNN belief-propagation decoder.
 *
 * This is the drop-in boundary for the reference's hot path (paths relative to
 * /root/reference/GNN-decode/):
 *
 *   MessagePassing.propagate()   quantum/decoder_v2_4.py:85-148, quantum/QGNNI.py:54-116,
 *                                quantum/BP.py:54-124, classical/CGNNI.py:52-112,
 *                                classical/BP.py:52-123       -> gnnd_propagate_tiled / _generic
 *   scatter_ (PyG-1.x)           quantum/decoder_v2_4.py:34-51 -> aggregation inside the above
 *   GNNI.forward() T-loop        classical/CGNNI.py:259-284, classical/BP.py:239-259,
 *     + update() MLPs + readout  quantum/BP.py:199-219, quantum/QGNNI.py:228-252,
 *                                quantum/decoder_v2_4.py:272-294 -> gnnd_decode
 *   H.to_sparse()._indices()     quantum/decoder_v2_4.py:164-165 -> gnnd_graph_create
 *
 * Conventions
 *   - Plain pointers and sizes only; no framework types.  Every pointer named d_* is DEVICE
 *     memory owned by the caller; h_* is host memory.  Kernels never allocate.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  No function that
 *     takes a stream synchronises the host, so every such call is graph-capturable.
 *   - Every function returns a gnnd_status; nothing throws or aborts.
 *   - Batch layout is the reference's PyG collation (graph-major): codeword b owns node rows
 *     [b*N, (b+1)*N) with N = V + C (variable rows first, then check rows) and edge rows
 *     [b*E, (b+1)*E) in the single-graph edge order (sorted by (v, c)).
 */
#ifndef GNND_H
#define GNND_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNND_VERSION 1

typedef enum gnnd_status {
    GNND_OK = 0,
    GNND_ERR_INVALID_ARG = 1,   /* bad pointer / size / enum value                     */
    GNND_ERR_HIP = 2,           /* a HIP runtime call failed (see gnnd_last_hip_error)  */
    GNND_ERR_UNSUPPORTED = 3,   /* valid request this build does not implement         */
    GNND_ERR_GRAPH = 4,         /* edge list is not a valid Tanner graph                */
    GNND_ERR_ALLOC = 5          /* device allocation failed (graph creation only)       */
} gnnd_status;

/* GNND_BF16 (gnnd_decode of CGNNI / CBP only): x and out stored as bf16 in HBM, weights
 * fp32 (gnnd_prepare_weights with GNND_F32), every operation in fp32 — BASELINE config 2's
 * "bf16" storage mode.                                                                      */
typedef enum gnnd_dtype { GNND_F32 = 0, GNND_F64 = 1, GNND_BF16 = 2 } gnnd_dtype;

/* `flow` of MessagePassing (quantum/decoder_v2_4.py:73-74,89):
 *   SOURCE_TO_TARGET: aggregate at edge_index[0] (variable nodes)  = v->c message
 *   TARGET_TO_SOURCE: aggregate at edge_index[1] (check nodes)     = c->v message     */
typedef enum gnnd_flow { GNND_SOURCE_TO_TARGET = 0, GNND_TARGET_TO_SOURCE = 1 } gnnd_flow;

/* `aggr` of MessagePassing (quantum/decoder_v2_4.py:70-71); PyG-1.x scatter_ rules. */
typedef enum gnnd_aggr { GNND_AGGR_ADD = 0, GNND_AGGR_MEAN = 1, GNND_AGGR_MAX = 2 } gnnd_aggr;

/* Which reference script's propagate body (the scripts each carry their own copy):
 *   V24    quantum/decoder_v2_4.py:132-144  c->v tanh(x/2); both flows cat extra[idx_j] (F=2)
 *   QGNNI  quantum/QGNNI.py:101-112         c->v tanh(x/2), cat (F=2); v->c + extra (F=1)
 *   QBP    quantum/BP.py:101-119            c->v log-domain BP with syndrome; v->c + extra
 *   CGNNI  classical/CGNNI.py:99-108        c->v tanh(x/2); + post (if non-NULL) (F=1)
 *   CBP    classical/BP.py:99-119           c->v log-domain BP; v->c + extra (F=1)
 *   NBP    quantum/neural_BP.py:108-131     c->v log-domain BP with syndrome, no +-10
 *                                           pre-clamp, p clamp 1 - 1e-15; v->c cat (F=2)
 *   V10    quantum/decoder_v1_0.py:109-131  c->v as NBP; v->c + extra (F=1)
 *   V30    quantum/decoder_v3_0.py:106-118  no pre-op on either side (edge states
 *                                           aggregated raw); both flows cat (F=2)
 *   V22    quantum/decoder_v2_2.py:133-160  the NBP body (the script's propagate is
 *                                           neural_BP.py's); decoder only: gnnd_propagate_*
 *                                           take NBP for it                              */
typedef enum gnnd_variant {
    GNND_V24 = 0, GNND_QGNNI = 1, GNND_QBP = 2, GNND_CGNNI = 3, GNND_CBP = 4,
    GNND_NBP = 5, GNND_V10 = 6, GNND_V30 = 7, GNND_V22 = 8
} gnnd_variant;

/* Whole-decoder models for gnnd_decode (same enumerators as gnnd_variant). */
typedef gnnd_variant gnnd_model;

typedef struct gnnd_graph gnnd_graph;   /* opaque; device-resident single-codeword graph */

/* ---- graph --------------------------------------------------------------------------
 * Build the single-codeword Tanner graph from its edge list, i.e. the reference's
 * `H.to_sparse()._indices()` of H[V, C] (row 0 = variable, row 1 = check), which must be
 * sorted by (v, c) with no duplicates.  Replaces the per-batch int64 edge_index reads of
 * the reference (quantum/decoder_v2_4.py:164-165, 277) with a cached CSR/CSC.          */
int gnnd_graph_create(const int64_t* h_var, const int64_t* h_chk, int64_t num_edges,
                      int32_t num_var, int32_t num_chk, gnnd_graph** out);
int gnnd_graph_destroy(gnnd_graph* g);
/* Host-only: build every table gnnd_graph_create would upload and check its structural
 * invariants (slot plans, padded / x-augmented message layouts); no device needed.
 * h_report4 = {slot plans checked, layouts checked, edges, invariant failures}.          */
int gnnd_graph_validate_host(const int64_t* h_var, const int64_t* h_chk, int64_t num_edges,
                             int32_t num_var, int32_t num_chk, int32_t* h_report4);
/* dims[0..5] = V, C, E, N, max variable degree, max check degree */
int gnnd_graph_dims(const gnnd_graph* g, int32_t* h_dims6);
/* Connected components the graph was split into (1 = not split).  A Tanner graph made of
 * 2..8 equal-shaped components, each a contiguous variable range with a contiguous check
 * range (the toric code of quantum/error_generate.py:39-132: its X and Z halves), is decoded
 * and trained by decoder_v2_4 with every component of a codeword in its own workgroup (the
 * components share no edge, so nothing is exchanged; results are the same as whole-graph
 * decoding up to fp32 summation order).  Set GNND_NO_SPLIT=1 to disable.                  */
int gnnd_graph_components(const gnnd_graph* g, int32_t* h_ncomp);
int gnnd_graph_set_split(gnnd_graph* g, int32_t enable);   /* 0: decode / train it whole */

/* Check on the device that a batched edge_index (int64, rows 0/1 at d_edge_index and
 * d_edge_index + row_stride, num_batched_edges columns) is the single graph tiled over
 * `batch` codewords with node offset b*N and check ids shifted by `chk_shift` (V after
 * GNNI.forward's shift, 0 before it).  Writes 1 (tiled) / 0 to *d_flag (device int32). */
int gnnd_check_tiled(const gnnd_graph* g, const int64_t* d_edge_index, int64_t row_stride,
                     int64_t num_batched_edges, int64_t batch, int64_t chk_shift,
                     int32_t* d_flag, void* stream);

/* ---- operator: one propagate() call ---------------------------------------------------
 * Tiled fast path (aggr ADD or MAX).  d_msg [B*E] (the per-edge `x` kwarg), d_extra [B*N]
 * (the `extra`/`post` argument; may be NULL only for CGNNI), d_out [B*E, F] row-major with
 * F = gnnd_propagate_width(variant, flow).  dtype selects float/double for all three.    */
int gnnd_propagate_width(int variant, int flow);
int gnnd_propagate_tiled(const gnnd_graph* g, int variant, int flow, int aggr, int dtype,
                         const void* d_msg, const void* d_extra, void* d_out, int64_t batch,
                         void* stream);

/* Generic path for an arbitrary edge_index (any aggr, including the reference's literal
 * leave-one-out `mean`).  Uses float atomics for the scatter, so sums are order-dependent
 * in the last bits.  d_workspace must hold gnnd_propagate_generic_workspace() bytes.    */
int gnnd_propagate_generic_workspace(int variant, int flow, int aggr, int dtype,
                                     int64_t num_edges, int64_t dim_size, int64_t* h_bytes);
int gnnd_propagate_generic(int variant, int flow, int aggr, int dtype,
                           const int64_t* d_edge_index, int64_t row_stride, int64_t num_edges,
                           const void* d_msg, const void* d_extra, int64_t dim_size,
                           void* d_out, void* d_workspace, int64_t workspace_bytes,
                           void* stream);

/* Backward of one propagate call w.r.t. d_msg (training; aggr ADD, every variant).
 * d_grad_out is [B*E, F] like d_out, d_grad_msg [B*E].  d_extra is the forward's `extra`
 * (the syndrome sets the sign of the BP check step; may be NULL except for the quantum BP
 * bodies QBP/NBP/V10 with flow TARGET_TO_SOURCE).  The c->v BP bodies recompute their
 * forward and apply torch's autograd rules (clamp passes the gradient on [lo, hi], abs
 * uses sign(t), tanh 1 - t^2).  The generic form needs a workspace of
 * gnnd_propagate_generic_bwd_workspace() bytes.                                           */
int gnnd_propagate_tiled_bwd(const gnnd_graph* g, int variant, int flow, int aggr, int dtype,
                             const void* d_msg, const void* d_extra, const void* d_grad_out,
                             void* d_grad_msg, int64_t batch, void* stream);
int gnnd_propagate_generic_bwd_workspace(int variant, int flow, int aggr, int dtype,
                                         int64_t num_edges, int64_t dim_size, int64_t* h_bytes);
int gnnd_propagate_generic_bwd(int variant, int flow, int aggr, int dtype,
                               const int64_t* d_edge_index, int64_t row_stride,
                               int64_t num_edges, const void* d_msg, const void* d_extra,
                               const void* d_grad_out, int64_t dim_size, void* d_grad_msg,
                               void* d_workspace, int64_t workspace_bytes, void* stream);

/* ---- fused T-iteration decoder --------------------------------------------------------
 * Runs the whole GNNI.forward (m0 = 0, T iterations of both half-steps, residual, readout)
 * for `batch` codewords in one launch; messages never leave the CU.
 *   d_x   [B*N]   node features (priors/LLRs at variable rows, syndrome at check rows)
 *   d_out [B*V]   P(bit = 1)  (sigmoid(-readout), clamped for the classical models)
 *         V30: [2*B*N], the reference's two-output readout (quantum/decoder_v3_0.py:
 *         274-290): [0, B*N) = sigmoid(-(mlp(S_v) + x)) per node (checks: S = 0),
 *         [B*N, 2*B*N) = sigmoid(-mlp(S_c(m_p))) per node (variables: S = 0), m_p = the
 *         v->c edge states of the last iteration
 *         V22: [iters*B*V], the reference's per-iteration readout list (quantum/
 *         decoder_v2_2.py:333-347): block t = sigmoid(-(S_v(m_t W) + S_v(x W_pr))) after
 *         iteration t (register-resident plans only: GNND_ERR_UNSUPPORTED otherwise)
 *   d_w   weights in `dtype` as produced by gnnd_prepare_weights from the packed
 *         state_dict layout below (gnnd_weights_count elements, same count after prepare):
 *     CGNNI: ggc2.mlp2 {W1[10], b1[10], W2[10], b2}, mlp {W1[10], b1[10], W2[10], b2}  = 62
 *     QGNNI: ggc2.mlp  {W1[10], b1[10], W2[10], b2}, mlp {same}                          = 62
 *     V24:   ggc1.mlp  {W1[:,0][128], W1[:,1][128], b1[128], W2[128], b2},
 *            ggc2.mlp  {W1[128], b1[128], W2[128], b2}, mlp {W1[128], b1[128], W2[128], b2}
 *                                                                                    = 1283
 *     CBP, QBP: none (d_w may be NULL)
 *     NBP (quantum/neural_BP.py, per-edge weights in reference edge order, T = iters):
 *            for t < T {layers[2t].W[E], layers[2t].W_p[E]}, then W[E], W_p[E], alpha
 *                                                                          = 2 E T + 2 E + 1
 *     V10 (quantum/decoder_v1_0.py): for t < T {layers[2t+1].W[E]}, then alpha  = E T + 1
 *     V22 (quantum/decoder_v2_2.py, weights shared by the 8 edge types of H_prime): the NBP
 *            layout with every type weight expanded per edge, w[e] = W[type(e)]:
 *            for t < T {layers[2t].W[type][E], layers[2t].W_p[type][E]}, then
 *            W[type][E], W_pr[type][E], sigmoid(weight)               = 2 E T + 2 E + 1
 *     V30 (quantum/decoder_v3_0.py, GRU edge states; the unused ggc1.mlp2/rnn2 and
 *            ggc2.mlp1/rnn1 are not passed):
 *            ggc1.mlp1 {W1[10][2] row-major, b1[10], W2[10], b2},
 *            ggc1.rnn1 {weight_ih[3], weight_hh[3], bias_ih[3], bias_hh[3]} (gates r, z, n),
 *            ggc2.mlp2 {same as ggc1.mlp1}, ggc2.rnn2 {same as rnn1},
 *            mlp {W1[10], b1[10], W2[10], b2}                                            = 137
 * gnnd_prepare_weights converts that layout into the kernel layout (for the fp32 V24
 * kernel the softplus layers are rescaled to base 2: layer-1 rows * log2(e), layer-2
 * weights * ln(2); V24 appends the check-MLP table and fp32 CGNNI / QGNNI the message
 * MLP's piecewise-linear table, gnnd_prepared_weights_count elements; every other model/dtype
 * is a plain copy).  Call it once per weights.
 * gnnd_weights_count is the graph-independent count (GNND_ERR_UNSUPPORTED for NBP/V10/V22,
 * whose packed layout is passed to gnnd_decode as is, without preparation);
 * gnnd_decode_weights_count covers every model for a graph and iteration count.         */
int gnnd_weights_count(int model, int64_t* h_count);
int gnnd_decode_weights_count(const gnnd_graph* g, int model, int32_t iters, int64_t* h_count);
int gnnd_prepare_weights(int model, int dtype, const void* d_w, void* d_prepared,
                         void* stream);
/* Elements of gnnd_prepare_weights' output: gnnd_weights_count, except V24 (7 264): the 1 283
 * weights (fp32: base-2 rescaled), then the check-MLP table (gnnd_v24_check_mlp_table) the
 * decoder and training forward read, then an 12-element channel-prior header (0 tables; see
 * gnnd_prepare_weights_priors), and fp32 CGNNI / QGNNI (328): the plain 62, then their message
 * MLP as a piecewise-linear table (<= 32 cells of <= 2 knots) the register-resident decoder
 * reads.  gnnd_decode needs this prepared buffer, not the plain weights (so does
 * gnnd_train_fwd for V24).                                                                  */
int gnnd_prepared_weights_count(int model, int dtype, int64_t* h_count);
int gnnd_decode(const gnnd_graph* g, int model, int dtype, const void* d_w, const void* d_x,
                void* d_out, int64_t batch, int32_t iters, void* stream);

/* Channel-prior tables (fp64 decoder_v2_4).  The variable-side MLP ggc1.mlp (Linear(2,128) ->
 * Softplus -> Linear(128,1), quantum/decoder_v2_4.py:237-239, :253-255) takes (S_v - m_e, x_v);
 * the reference's inputs carry one prior LLR x_v = log((1-p)/p) per codeword, p drawn from a
 * short list (quantum/error_generate.py:252-260).  gnnd_prepare_weights_priors = gnnd_prepare_weights
 * plus, for each of the n_priors values h_priors[] (host fp64, <= 64; the exact x_v bits the
 * inputs will carry), tanh(MLP/2) -- the check step's pre-op of its output -- tabulated over
 * |S_v - m_e| <= 32 (64-byte cells: degree-7 Taylor polynomials about j/16; the readout MLP's
 * about j/32; up to 3 units crossing torch's Softplus threshold inside a cell are stored aside and
 * their jumps added exactly; a cell whose MLP remainder bound exceeds 1e-13, whose tanh series
 * misses tanh(P/2) of the MLP's own cell polynomial P at a cell edge by more than 2e-14, or that
 * holds more crossings is marked invalid and its points take the 128 units), into a buffer of
 * gnnd_prepared_weights_count_priors elements.  gnnd_decode
 * (fp64 V24, batches decoded one wave per item group) then reads a codeword's table where its
 * x_v equals a registered prior bit for bit and evaluates the 128 units elsewhere (other priors,
 * |S_v - m_e| > 32), and the readout MLP from one more table (n_priors > 0).  The tables
 * depend on the weights: gnnd_train_update and
 * gnnd_prepare_weights reset the count to 0.  Other models/dtypes: n_priors must be 0.        */
int gnnd_prepared_weights_count_priors(int model, int dtype, int32_t n_priors, int64_t* h_count);
int gnnd_prepare_weights_priors(int model, int dtype, const void* d_w, void* d_prepared,
                                const double* h_priors, int32_t n_priors, void* stream);
/* The tables as the decoder evaluates them, for tests: d_y[i] = tanh(ggc1.mlp(d_u[i], d_x[i]) / 2)
 * (the prior tables hold the check step's pre-op tanh(m/2) of ggc1's output directly, as degree-7
 * series composed from the MLP's; quantum/decoder_v2_4.py:135-136) and
 * d_hit[i] = 1 where a table covers the point, else d_hit[i] = 0 and d_y[i] untouched
 * (d_w = prepared fp64 V24 weights with tables; device fp64 d_u, d_x, d_y [n], int32 d_hit).
 * The prepared tables end with one for the readout MLP (mlp, quantum/decoder_v2_4.py:291, over
 * |m| <= 32, no prior): d_x = NULL evaluates that one, d_y[i] = mlp(d_u[i]).                 */
int gnnd_v24_var_mlp_table(const void* d_w, const void* d_u, const void* d_x, void* d_y,
                           int32_t* d_hit, int64_t n, void* stream);

/* decoder_v2_4's check-side MLP (ggc2.mlp: Linear(1,128) -> Softplus -> Linear(128,1),
 * quantum/decoder_v2_4.py:241-243, :253-257) as the fp64 decoder evaluates it: its input
 * u = S_c(tanh(m/2)) - tanh(m_e/2) lies in [-R, R], R = max check degree - 1, so the fp64
 * prepared weights carry it tabulated (degree-11 Taylor polynomials about j/8, |j/8| <= 31;
 * gnnd_prepare_weights and gnnd_train_update build the table) and the decoder reads the table
 * instead of the 128 hidden units.  This evaluates the same table at d_u [n] (fp64, inside
 * [-R, R]) into d_y [n]; d_w = PREPARED fp64 V24 weights.  *d_ok (device int32) = 1 when the
 * table is valid for this graph -- the decoder uses it -- or 0 (d_y untouched) when a unit's
 * pre-activation crosses torch's Softplus threshold 20 for some u in [-R, R], the Taylor
 * remainder bound exceeds 1e-13, or R > 31 (the decoder then evaluates the units).          */
int gnnd_v24_check_mlp_table(const gnnd_graph* g, const void* d_w, const void* d_u, void* d_y,
                             int64_t n, int32_t* d_ok, void* stream);

/* Codewords per workgroup the decoder would use (for roofline bookkeeping). */
int gnnd_decode_tile(const gnnd_graph* g, int model, int dtype, int32_t* h_cw_per_block,
                     int32_t* h_lds_bytes);
/* Full launch plan: h_plan[0] codewords per workgroup, [1] LDS bytes per workgroup,
 * [2] kernel (0 = streaming decode_kernel, 1 = register-resident decode_resident_kernel),
 * [3] work items per lane (resident kernel; 0 otherwise), [4] variable-sum group of the
 * resident kernel's message layout (vars per wave step padded to one degree; 1 = identity
 * layout; 0 for the streaming kernel).  h_plan holds 5 ints. */
int gnnd_decode_plan(const gnnd_graph* g, int model, int dtype, int32_t* h_plan);

/* ---- fused training step (decoder_v2_4) ------------------
 * gnnd_train_fwd = gnnd_decode (same prepared weights, same output) that also writes the
 * training tape (gnnd_train_tape_bytes bytes of d_tape): per iteration and edge the
 * v->c MLP input, the tanh output and the c->v MLP input, plus the final messages.
 * gnnd_train_bwd turns d loss / d out [B*V] into d loss / d weights [1283] (V24) in the PLAIN
 * packed layout of gnnd_weights_count (d_w is that plain layout, not the prepared one):
 * reverse mode through all T iterations and the readout in one launch (+ a fixed-order
 * reduction of per-workgroup partials in d_workspace, gnnd_train_bwd_workspace bytes).
 * Models: V24 (quantum/decoder_v2_4.py:260-294, fp32/fp64), V30 (quantum/decoder_v3_0.py:
 * 245-290, fp32/fp64; d_out / d_grad_out are the two readout tensors [2][B*N]), and fp64 NBP
 * (quantum/neural_BP.py:263-314), V22 (quantum/decoder_v2_2.py:299-347; d_out /
 * d_grad_out every layer's readout [T][B*V]) and V10 (quantum/decoder_v1_0.py:263-313)
 * whose gradient is w.r.t. the per-edge tables of their packed layout (NBP/V22 2 E T + 2 E + 1
 * values, V10 E T + 1), CGNNI (classical/CGNNI.py:248-284) and
 * QGNNI (quantum/QGNNI.py:217-252), fp32/fp64, gradient w.r.t. their 62 packed weights (the
 * forward writes its own tape: every iteration's tanh outputs and the readout inputs; d_out
 * is its prediction, not gnnd_decode's register-resident one bit for bit).  The other models
 * train through gnnd_propagate_*_bwd.  gnnd_train_workspace_bytes sizes the workspace of every model
 * (gnnd_train_bwd_workspace, which has no iteration count, only V24 and V30).             */
int gnnd_train_tape_bytes(const gnnd_graph* g, int model, int dtype, int64_t batch,
                          int32_t iters, int64_t* h_bytes);
int gnnd_train_fwd(const gnnd_graph* g, int model, int dtype, const void* d_w, const void* d_x,
                   void* d_out, void* d_tape, int64_t batch, int32_t iters, void* stream);
int gnnd_train_bwd_workspace(const gnnd_graph* g, int model, int dtype, int64_t batch,
                             int64_t* h_bytes);
int gnnd_train_workspace_bytes(const gnnd_graph* g, int model, int dtype, int64_t batch,
                               int32_t iters, int64_t* h_bytes);
int gnnd_train_bwd(const gnnd_graph* g, int model, int dtype, const void* d_w, const void* d_x,
                   const void* d_out, const void* d_grad_out, const void* d_tape,
                   void* d_grad_w, void* d_workspace, int64_t workspace_bytes, int64_t batch,
                   int32_t iters, void* stream);
/* The reverse pass without its reduction: leaves gnnd_train_bwd_rows() per-workgroup
 * gradient rows [rows][n] (n = the model's weights: V24 1283, V30 137, CGNNI/QGNNI 62,
 * NBP/V22 2ET + 2E + 1, V10 ET + 1) in d_workspace, for gnnd_train_update (V24, V30, CGNNI, QGNNI) to
 * reduce (fused with
 * the optimizer).  On a split graph (gnnd_graph_components > 1) every component of a
 * codeword runs in its own workgroup.                                                     */
int gnnd_train_bwd_rows(const gnnd_graph* g, int model, int dtype, int64_t batch,
                        int64_t* h_rows);
int gnnd_train_bwd_partial(const gnnd_graph* g, int model, int dtype, const void* d_w,
                           const void* d_x, const void* d_out, const void* d_grad_out,
                           const void* d_tape, void* d_workspace, int64_t workspace_bytes,
                           int64_t batch, int32_t iters, void* stream);
/* The reverse pass with the syndrome loss of gnnd_syndrome_loss fused in: d_y [B*V] labels,
 * d_logical_mask [V] uint32 = bit l set iff variable v is in logical row l (n_logical <= 32;
 * on a split graph every row's support must lie inside one component).  Each workgroup
 * computes the loss terms of its codeword (component) and their gradient itself; the losses
 * go to d_loss_b [gnnd_train_loss_count(batch)] (one per codeword and component, in codeword
 * order); the batch loss is their sum (gnnd_train_update sums them).  Rows as
 * gnnd_train_bwd_partial.                                                                  */
int gnnd_train_loss_count(const gnnd_graph* g, int64_t batch, int64_t* h_count);
int gnnd_train_bwd_loss_partial(const gnnd_graph* g, int model, int dtype, const void* d_w,
                                const void* d_x, const void* d_out, const void* d_y,
                                const uint32_t* d_logical_mask, int32_t n_logical,
                                int32_t logical_only, const void* d_tape, void* d_loss_b,
                                void* d_workspace, int64_t workspace_bytes, int64_t batch,
                                int32_t iters, void* stream);
/* The same syndrome loss computed in the FORWARD's epilogue instead: gnnd_train_fwd plus
 * d_grad_out [B*V] = d loss / d out and d_loss_b as above (the same terms and summation
 * orders, so the same bits), for gnnd_train_bwd_partial(d_grad_out) to consume.  fp32 V24
 * on its unit-split small-batch plan only (the 16-wave reverse pass then skips its loss
 * phases); returns GNND_ERR_UNSUPPORTED (nothing launched) otherwise.                       */
int gnnd_train_fwd_loss(const gnnd_graph* g, int model, int dtype, const void* d_w,
                        const void* d_x, void* d_out, void* d_tape, const void* d_y,
                        const uint32_t* d_logical_mask, int32_t n_logical, int32_t logical_only,
                        void* d_grad_out, void* d_loss_b, int64_t batch, int32_t iters,
                        void* stream);
/* Fused optimizer epilogue of a decoder_v2_4 training step (one launch):
 *   n_rows > 0: d_grad[i] = fixed-order sum of the rows (d_grad may be NULL: not stored);
 *   n_rows = 0: the gradient is read from d_grad (e.g. after an all-reduce of it);
 *   d_loss_b [batch] non-NULL: *d_loss = fixed-order sum of the per-codeword losses;
 *   d_param non-NULL: gnnd_adam_step's update of the plain packed weights (V24 1283, V30 137,
 *   CGNNI/QGNNI 62; the V30, CGNNI and QGNNI kernel layouts are the plain one) (moments
 *   d_exp_avg / d_exp_avg_sq, device step count *d_step incremented once), then, if
 *   d_prepared is non-NULL, gnnd_prepare_weights' kernel layout of the updated weights into
 *   d_prepared.  d_sync: one device uint32, zero before the first call (the kernel leaves it
 *   zero); it orders the step-count update across the launch's workgroups.
 * Single-rank step: bwd_partial -> update(rows, loss, Adam, prepare).  Data-parallel step:
 * bwd_partial -> update(rows -> d_grad, loss) -> all_reduce(d_grad) -> update(0 rows, Adam). */
int gnnd_train_update(int model, int dtype, const void* d_rows, int64_t n_rows, void* d_grad,
                      const void* d_loss_b, int64_t batch, void* d_loss, void* d_param,
                      void* d_exp_avg, void* d_exp_avg_sq, double* d_step, uint32_t* d_sync,
                      double lr, double beta1, double beta2, double eps, double weight_decay,
                      void* d_prepared, void* stream);

/* ---- training objective ------------------------------------------------
 * Syndrome loss of quantum/decoder_v2_4.py:297-317 (logical_only != 0: the Lambda term of
 * quantum/QGNNI.py:255-290 only) and its gradient, per codeword b of the batch:
 *   d_loss_b[b] = sum_c |sin(pi/2 (H^T (y+p))_c)| + sum_l |sin(pi/2 (Lambda (y+p))_l)|
 *   d_dpred[b*V+v] = d loss_b / d p_v  (torch's |.| rule: sign(0) = 0)
 * d_pred, d_y: [B*V] in dtype; d_logical: int32 [n_logical][V] 0/1 rows of Lambda.  The
 * batch loss of the reference is sum_b d_loss_b[b].  Replaces the reference's LossFunc
 * (its O(B) torch.cat reshape loop and ~30 small autograd kernels per step).            */
int gnnd_syndrome_loss(const gnnd_graph* g, const int32_t* d_logical, int32_t n_logical,
                       int32_t logical_only, int dtype, const void* d_pred, const void* d_y,
                       void* d_loss_b, void* d_dpred, int64_t batch, void* stream);

/* Hard-decision metrics of a decoded batch, replacing the O(B) torch.cat
 * loops of quantum/neural_BP.py:333-348 (FER rule) and the host-side BER counts:
 *   e = (pred > 0.5) xor (y > 0.5) per bit;
 *   d_counts[0] = sum of e (bit errors), [1] = codewords with any bit error,
 *   [2] = codewords with a nonzero residual syndrome H^T e,
 *   [3] = codewords with zero residual syndrome and an odd overlap with some logical row.
 * d_pred, d_y: [B*V] in dtype; d_logical: int32 [n_logical][V] 0/1 rows (n_logical = 0 for
 * classical codes); d_counts: 4 int64 on the device (overwritten).                        */
int gnnd_decision_errors(const gnnd_graph* g, const int32_t* d_logical, int32_t n_logical,
                         int dtype, const void* d_pred, const void* d_y, int64_t* d_counts,
                         int64_t batch, void* stream);

/* Adam (torch.optim.Adam update order, amsgrad/maximize off) on one flat parameter buffer of
 * n values with its two moment buffers; *d_step is the device-resident step count (double,
 * incremented by the call), so a whole training step with the update can be captured in one
 * HIP graph.  Single-workgroup kernel (sized for the decoders' ~10^3 parameters).          */
int gnnd_adam_step(int dtype, void* d_param, const void* d_grad, void* d_exp_avg,
                   void* d_exp_avg_sq, double* d_step, int64_t n, double lr, double beta1,
                   double beta2, double eps, double weight_decay, void* stream);

/* ---- input synthesis ---------------------------------------------------
 * Decoder inputs in the batch layout above, generated on the device with Philox4x32-10
 * (counter = {word, global codeword index lo/hi, stream}, key = seed): codeword b of the
 * call is global codeword offset + b, so data-parallel shards passing offset = shard start
 * draw exactly the codewords one single-device call over the global batch would.
 *   gnnd_sample_toric  quantum/error_generate.py:252-278 (gen_syn): p uniform over h_p[n_p]
 *     (n_p <= 16) per codeword, every variable flips with probability p; d_x [B*N] =
 *     {log((1-p)/p) at variable rows, (-1)^(H^T e) at check rows}, d_y [B*V] = e.
 *   gnnd_sample_awgn   classical/CGNNI.py:125-147 (Gen_Data.AWGN, get_post): codeword =
 *     the constant word codeword_bit (d_gen_cols NULL) or m G for k uniform message bits,
 *     d_gen_cols [V][ceil(k/32)] uint32 = the generator's columns as bit masks; BPSK
 *     1 - 2c, sigma^2 = 10^(-SNR/10) with SNR = h_snr_db[(offset + b) % n_snr] (n_snr <= 16);
 *     d_x [B*N] = {2 y' / sigma^2 at variable rows, 0 at check rows}, d_y [B*V] = c.
 * gnnd_philox4x32_10 is the host mirror of the generator (known-answer tests).            */
int gnnd_sample_toric(const gnnd_graph* g, int dtype, const double* h_p, int32_t n_p,
                      uint64_t seed, int64_t offset, void* d_x, void* d_y, int64_t batch,
                      void* stream);
int gnnd_sample_awgn(const gnnd_graph* g, int dtype, const double* h_snr_db, int32_t n_snr,
                     const uint32_t* d_gen_cols, int32_t k, int32_t codeword_bit, uint64_t seed,
                     int64_t offset, void* d_x, void* d_y, int64_t batch, void* stream);
void gnnd_philox4x32_10(const uint32_t* h_ctr4, const uint32_t* h_key2, uint32_t* h_out4);

/* ---- debug build (make debug -> libgnnd_debug.so, -DGNND_DEBUG) ----------------------------
 * The kernels check the table-derived indices they otherwise trust and record violations
 * as bits (0 LDS position, 1 variable id, 2 slot, 3 node, 4 grid) instead of faulting;
 * gnnd_debug_flags synchronises the device and returns (and clears) their OR.  In release
 * builds gnnd_debug_enabled() is 0 and the flags are always 0.                             */
int gnnd_debug_enabled(void);
int gnnd_debug_flags(uint32_t* h_flags);

/* ---- misc ----------------------------------------------------------------------------- */
const char* gnnd_status_string(int status);
int gnnd_last_hip_error(void);          /* hipError_t of the last GNND_ERR_HIP, per thread */
int gnnd_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GNND_H */
