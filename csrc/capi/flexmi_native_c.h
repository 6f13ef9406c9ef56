/* flexmi NATIVE C API: flexmi's C++ runtime from C without any Python.
 *
 * flexmi_c.h is the CPython-embedding model API (it drives the Python front end through an
 * embedded interpreter, like the reference's cffi layer drives its C++ core).  This header is the
 * CPython-free layer over the native runtime itself (libflexmi_native_c.so links only the C++
 * runtime): the native plan compiler and trainer (fmn_model_*: dense / embedding / dot-interaction
 * DLRM graphs and convolution / pooling CNN graphs under data, table-, column-, row- and
 * channel-parallel plans, CPU and HIP engines), strategy files in the reference's protobuf format,
 * the sharding algebra of the plan
 * compiler (partitions, boxes, reshard transfer lists), the MI355X execution simulator and MCMC
 * SOAP search, the HDF5 dataset reader, the prefetching batch loader ring and the CPU
 * embedding-bag kernels.  Reference counterparts: src/runtime/strategy.cc (.pb files),
 * src/runtime/simulator.cc + model.cc:1082-1144 (simulate / optimize), python/flexflow_dataloader.cc
 * (loaders), src/ops/embedding.cc:87-163 / embedding_avx2.cc (CPU embedding).
 *
 * Conventions: handles are opaque; functions return NULL / a negative value on error and the
 * message is available from fmn_last_error() (thread-local).  Boxes are [lo, hi) per dim,
 * passed as lo[nd] / hi[nd] arrays.
 */
#ifndef FLEXMI_NATIVE_C_H
#define FLEXMI_NATIVE_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fmn_strategy_s* fmn_strategy_t;
typedef struct fmn_layout_s* fmn_layout_t;
typedef struct fmn_sim_s* fmn_sim_t;
typedef struct fmn_h5_s* fmn_h5_t;
typedef struct fmn_loader_s* fmn_loader_t;
typedef struct fmn_plan_s* fmn_plan_t;

const char* fmn_last_error(void);
const char* fmn_version(void);

/* ---- strategy files (reference .pb format: name, device type, dims, device ids) ----------- */
fmn_strategy_t fmn_strategy_create(void);
fmn_strategy_t fmn_strategy_load(const char* path);
int fmn_strategy_save(fmn_strategy_t s, const char* path);
void fmn_strategy_destroy(fmn_strategy_t s);
int fmn_strategy_num_ops(fmn_strategy_t s);
/* index of op `name`, -1 if absent */
int fmn_strategy_find(fmn_strategy_t s, const char* name);
/* op i: name (truncated to len), device type (0 GPU, 1 CPU), dims (reference order: innermost
 * first, sample dim last), device ids; returns the number of parts (product of dims) */
int fmn_strategy_get(fmn_strategy_t s, int i, char* name, size_t len, int* device_type, int* ndims, int* dims, int max_dims,
                     int* ndev, int* devs, int max_devs);
/* add or replace op `name` */
int fmn_strategy_set(fmn_strategy_t s, const char* name, int device_type, int ndims, const int* dims, int ndev,
                     const int* devs);

/* ---- sharding algebra ---------------------------------------------------------------------- */
/* [lo, hi) of block k of n split into d near-equal blocks */
int fmn_split_extent(int64_t n, int64_t d, int64_t k, int64_t* lo, int64_t* hi);
/* a layout: shape[nd], degrees[nd] (user order, outer -> inner); part p is held by holders[p]
 * (one rank each; replicate with fmn_layout_add_holder) */
fmn_layout_t fmn_layout_create(int nd, const int64_t* shape, const int64_t* degrees, const int* holders, int partial);
int fmn_layout_add_holder(fmn_layout_t l, int part, int rank);
int64_t fmn_layout_num_parts(fmn_layout_t l);
int fmn_layout_part_box(fmn_layout_t l, int64_t part, int64_t* lo, int64_t* hi);
void fmn_layout_destroy(fmn_layout_t l);
/* transfers turning src into dst (sorted by src, dst, dst_part, src_part, box): returns the
 * count; the first max_n are written (src, dst ranks; boxes as nd-wide lo / hi rows) */
int fmn_reshard_transfers(fmn_layout_t src, fmn_layout_t dst, int max_n, int* src_rank, int* dst_rank, int64_t* lo,
                          int64_t* hi);

/* ---- MI355X simulator + MCMC SOAP search ----------------------------------------------------- */
/* ndev GPUs, gpus_per_node per node; link_GBps / ar_busbw_GBps <= 0 keep the MI355X defaults */
fmn_sim_t fmn_sim_create(int ndev, int gpus_per_node, double link_GBps, double ar_busbw_GBps);
void fmn_sim_destroy(fmn_sim_t s);
/* tensor: element bytes, producer op (-1 = graph input) and its output index */
int fmn_sim_add_tensor(fmn_sim_t s, int elem_bytes, int producer, int producer_out, int needs_grad);
/* op with inputs / outputs (tensor ids); candidates are added next, in order */
int fmn_sim_add_op(fmn_sim_t s, const char* name, int n_in, const int* in_t, int n_out, const int* out_t);
/* candidate of the last added op: parts on devices part_dev[nparts] with per-part fwd / bwd us;
 * output / needed-input layouts per tensor as nparts boxes (nd-wide lo / hi rows, each part held
 * by its own device), replicated-weight gradient bytes (all-reduced over the part devices when
 * > 0) and per-part memory bytes.  Returns the candidate index. */
int fmn_sim_add_candidate(fmn_sim_t s, int nparts, const int* part_dev, const double* fwd_us, const double* bwd_us, int nd,
                          const int64_t* out_lo, const int64_t* out_hi, const int64_t* in_lo, const int64_t* in_hi,
                          double wsync_bytes, double mem_bytes, const char* label);
/* makespan (us) of one training iteration for candidate choice assign[num_ops] */
double fmn_sim_simulate(fmn_sim_t s, const int* assign);
/* Metropolis search from init[num_ops] for `budget` proposals: writes best[num_ops], returns
 * its simulated time (us) */
double fmn_sim_search(fmn_sim_t s, const int* init, long budget, double alpha, uint64_t seed, int* best);

/* ---- HDF5 datasets (the DLRM --dataset files) ------------------------------------------------ */
fmn_h5_t fmn_h5_open(const char* path);
void fmn_h5_close(fmn_h5_t h);
int fmn_h5_num_datasets(fmn_h5_t h);
/* dataset i: name, numpy dtype string ("<f4", "<i8", ...), rank / shape; returns 0 */
int fmn_h5_dataset_info(fmn_h5_t h, int i, char* name, size_t name_len, char* dtype, size_t dtype_len, int* ndims,
                        int64_t* shape, int max_dims);
/* copy rows [row0, row0 + nrows) of dataset `name` (row = product of the trailing dims) into dst */
int64_t fmn_h5_read_rows(fmn_h5_t h, const char* name, int64_t row0, int64_t nrows, void* dst, size_t dst_bytes);

/* ---- batch loader ring (host threads gather batches ahead of the training loop) --------------- */
fmn_loader_t fmn_loader_create(int64_t batch, int64_t num_samples, int depth, int threads, int shuffle, uint64_t seed);
/* a source: full dataset base[rows][row_bytes]; this rank copies bytes [col_off, col_off +
 * col_bytes) of rows [row_lo, row_hi) of every batch into its staging slots (pitch dst_pitch) */
int fmn_loader_add_source(fmn_loader_t l, const void* base, int64_t rows, int64_t row_bytes, int64_t col_off,
                          int64_t col_bytes, int64_t row_lo, int64_t row_hi, int64_t dst_pitch);
int fmn_loader_set_slot(fmn_loader_t l, int source, int slot, void* ptr);
int fmn_loader_start(fmn_loader_t l);
int fmn_loader_acquire(fmn_loader_t l);           /* next batch's slot (blocks) */
int fmn_loader_release(fmn_loader_t l, int slot);
int64_t fmn_loader_batches_per_epoch(fmn_loader_t l);
int fmn_loader_batch_ids(fmn_loader_t l, int64_t n, int64_t* ids, int64_t max_ids);
void fmn_loader_destroy(fmn_loader_t l);

/* ---- graph planner (csrc/runtime/planner.h) ----------------------------------------------------
 * Build the graph op by op (model order; the loss reads the first output of the LAST op), then
 * plan: communication-first order, forward reshard schedule, backward liveness and schedule. */
fmn_plan_t fmn_plan_create(void);
/* returns the op index; outputs are tensor ids */
int fmn_plan_add_op(fmn_plan_t p, int64_t guid, int n_out, const int64_t* outputs);
/* adds an input to the last op: flags bit 0 is_float, 1 needs_grad, 2 reshard, 3 remote */
int fmn_plan_add_input(fmn_plan_t p, int64_t tensor, int64_t producer, int dtype, int64_t need, int flags);
int fmn_plan_run(fmn_plan_t p, int world, int input_grads);
/* results (after fmn_plan_run): counts and copies; steps are (kind, op guid, #inputs) rows whose
 * input indices follow in `inputs` (kind: 0 op, 1 reshard (fwd) / gradient reduce (bwd)) */
int64_t fmn_plan_order(fmn_plan_t p, int64_t* guids, int64_t max_n);
int64_t fmn_plan_bwd_live(fmn_plan_t p, int64_t* guids, int64_t max_n);
int64_t fmn_plan_grad_needed(fmn_plan_t p, int64_t* tensors, int64_t max_n);
int64_t fmn_plan_steps(fmn_plan_t p, int backward, int* kind, int64_t* op, int* n_inputs, int* inputs, int64_t max_steps,
                       int64_t max_inputs);
void fmn_plan_destroy(fmn_plan_t p);

/* ---- CPU embedding-bag kernels --------------------------------------------------------------- */
/* out[b * ld_out + d] = scale * sum_j W[idx[b * bag + j] - row_lo][d] (rows outside the shard skipped) */
int fmn_embedding_bag_forward(const float* W, int64_t rows, int64_t D, const int64_t* idx, int64_t B, int64_t bag,
                              int64_t row_lo, float scale, float* out, int64_t ld_out);
/* target[idx[b * bag + j] - row_lo][d] += alpha * dy[b * ld_dy + d]  (gradient: alpha = scale;
 * fused sparse SGD on the table: alpha = -lr * scale) */
int fmn_embedding_bag_backward(float* target, int64_t rows, int64_t D, const int64_t* idx, int64_t B, int64_t bag,
                               int64_t row_lo, const float* dy, int64_t ld_dy, float alpha);

/* ---- native model: build, plan and train an MLP or a DLRM entirely in C++ -------------------------
 * The plan compiler (csrc/runtime/native_model.cc) lays out one rank's buffers: data parallelism
 * for the dense layers (sample split; replicated weights in one flat buffer; gradient all-reduce
 * buckets in backward order) and TABLE-WISE model parallelism for embedding tables (each table
 * whole on one rank, global-batch lookups there, an all-to-all to the sample shards and back,
 * sparse SGD of the touched rows on the owner); it decides the fused epilogues and runs the step
 * on an engine: device 0 = CPU (reference fp32 loops; `world` rank PROCESSES exchange through a
 * shared mapping in the `rendezvous` directory), device 1 = HIP (flexmi's gfx950 kernels from
 * libflexmi_kernels.so, RCCL across `world` processes that share the `rendezvous` directory).
 * Reference: FFModel compile / init_layers / forward / backward / update (src/runtime/model.cc),
 * the DLRM app and strategy (examples/cpp/DLRM/dlrm.cc, src/runtime/dlrm_strategy.cc). */
typedef struct fmn_model_s* fmn_model_t;
fmn_model_t fmn_model_create(int global_batch, int device, int rank, int world, const char* rendezvous);
void fmn_model_destroy(fmn_model_t m);
/* tensor ids: the input (features per sample), then a chain of dense layers (act: 10 none,
 * 11 relu, 12 sigmoid, 13 tanh) */
int fmn_model_input(fmn_model_t m, int features);
int fmn_model_dense(fmn_model_t m, int input_tensor, int out_dim, int activation, int use_bias);
/* CNN graphs (data parallel): an image input [B][C][H][W] (NCHW, train_step takes the global batch
 * of C*H*W features per sample), 2-D convolutions (out channels, kernel, stride, symmetric zero
 * padding, fused bias + activation) and poolings (is_max 1: max, 0: average excluding the
 * padding) -> their [B][C'][P][Q] tensor ids; dense layers take them flattened.  Reference:
 * FFModel::conv2d / pool2d (include/model.h, src/ops/conv_2d.cu, src/ops/pool_2d.cu). */
int fmn_model_input_image(fmn_model_t m, int channels, int height, int width);
int fmn_model_conv2d(fmn_model_t m, int input_tensor, int out_channels, int kernel_h, int kernel_w, int stride_h,
                     int stride_w, int pad_h, int pad_w, int activation, int use_bias);
int fmn_model_pool2d(fmn_model_t m, int input_tensor, int kernel_h, int kernel_w, int stride_h, int stride_w, int pad_h,
                     int pad_w, int is_max);
/* batch norm of an image tensor (training-mode statistics over this rank's samples, scale 1 / bias 0
 * at init, optional fused ReLU); returns the output tensor id */
int fmn_model_batch_norm(fmn_model_t m, int input_tensor, int relu);
/* DLRM graphs: a sparse input (int64 [B][bag] lookup indices of the GLOBAL batch) -> its id; an
 * embedding table rows x dim over a sparse input (SUM bag) -> its [B][dim] tensor id; the dot
 * interaction of a bottom tensor and n embedding tensors -> its [B][W] tensor id (W = dim +
 * F(F-1)/2 padded to pad_to).  Every tensor has one consumer. */
int fmn_model_sparse_input(fmn_model_t m, int bag);
int fmn_model_embedding(fmn_model_t m, int sparse_input, int64_t rows, int dim);
int fmn_model_dot_interaction(fmn_model_t m, int bottom, int n, const int* embeddings, int pad_to);
/* place table t (embedding creation order) on `rank` (before compile; default: greedy by rows) */
int fmn_model_set_table_owner(fmn_model_t m, int table, int rank);
int fmn_model_table_owner(fmn_model_t m, int table);
/* column split of a table over n holder ranks (dim % n == 0): holder j keeps columns [j*dim/n,
 * (j+1)*dim/n); set/get_param of such a table move the FULL rows x dim host array (this rank's
 * columns read / written).  fmn_model_table_columns returns the holder count (after compile: 1 for
 * a table-wise table) and writes up to max holder ranks. */
int fmn_model_set_table_columns(fmn_model_t m, int table, int n, const int* ranks);
int fmn_model_table_columns(fmn_model_t m, int table, int* ranks, int max);
/* row split of a table over n holder ranks: holder j keeps rows [j*rows/n, (j+1)*rows/n) of every
 * column, looks up the global batch (lookups outside its rows add nothing) and each rank sums the
 * holders' partial bag sums; set/get_param move the FULL host array (this rank's rows). */
int fmn_model_set_table_rows(fmn_model_t m, int table, int n, const int* ranks);
/* channel split of dense layer `layer` (creation order among the dense layers) over n holder ranks:
 * holder j keeps output features [j*N/n, (j+1)*N/n) and computes them for the global batch (input
 * gathered, outputs and input gradients exchanged by all-to-all, its slice updated without an
 * all-reduce); set/get_param move the FULL W [N][K] / b [N] host arrays (this rank's slice). */
int fmn_model_set_dense_channels(fmn_model_t m, int layer, int n, const int* ranks);
/* place the model's dense layers / tables by a strategy (e.g. the MCMC search's result saved as a
 * .pb): dense layer i is op dense_names[i], table t is op table_names[t] (NULL names: skipped).
 * Internal dims (reference order, dim 0 fastest in the device list): Linear [c, n] -> channel split
 * over the devices of channel slices 0..c-1 (c = 1 and one part: the layer on that device; else
 * data parallel); Embedding [c, n] or [c, n, r] -> column split over c devices, row split over r
 * devices, or the table on device 0 of the list.  A config the native plan cannot express exactly
 * (uneven channels, a device repeated) falls back to data parallel / table-wise, which computes the
 * same values.  Returns the number of ops placed from the strategy. */
int fmn_model_apply_strategy(fmn_model_t m, fmn_strategy_t s, int n_dense, const char* const* dense_names, int n_tables,
                             const char* const* table_names);
/* optimizer of the dense parameters (before compile; default plain SGD): type 0 SGD at compile's lr
 * with momentum / Nesterov / weight decay, 1 Adam with alpha = compile's lr (beta1, beta2, epsilon,
 * weight decay).  A model with embedding tables needs plain SGD (its tables take sparse in-place
 * updates).  Reference: SGDOptimizer / AdamOptimizer (include/optimizer.h, src/runtime/optimizer.cc). */
int fmn_model_set_optimizer(fmn_model_t m, int type, float momentum, int nesterov, float weight_decay, float beta1,
                            float beta2, float epsilon);
/* ZeRO stage 1 (before compile; world > 1): gradient buckets reduce-scattered, the optimizer state of
 * the data-parallel parameters kept for this rank's 1/world slice of each bucket, the updated slices
 * all-gathered.  0 turns it off. */
int fmn_model_set_zero(fmn_model_t m, int stage);
/* loss: 51 sparse categorical CE (softmax of the last layer's logits, int32 labels), 52 MSE (avg),
 * 54 binary CE (sigmoid output); bucket_mb = gradient all-reduce bucket size */
int fmn_model_compile(fmn_model_t m, int loss_type, float lr, double bucket_mb);
int fmn_model_init_weights(fmn_model_t m, uint64_t seed);
/* parameter entries in model order: weight [out][in] then bias [out] of every dense layer, the
 * [rows][dim] table of every embedding; a table is readable / writable on its owner only
 * (fmn_model_param_local) */
int fmn_model_num_params(fmn_model_t m);
int64_t fmn_model_param_numel(fmn_model_t m, int i);
int fmn_model_param_local(fmn_model_t m, int i);
int fmn_model_set_param(fmn_model_t m, int i, const float* host);
int fmn_model_get_param(fmn_model_t m, int i, float* host);
/* one training step on the GLOBAL batch x [B][features] (each rank takes its sample shard) and
 * labels ([B] int32 for loss 51, [B][out] float otherwise); loss = this rank's mean loss */
int fmn_model_train_step(fmn_model_t m, const float* x, const void* labels, double* loss, int64_t* correct);
/* the same with the sparse inputs: sparse[s] = GLOBAL [B][bag] int64 indices of sparse input s */
int fmn_model_train_step_sparse(fmn_model_t m, const float* x, const int64_t* const* sparse, const void* labels,
                                double* loss, int64_t* correct);
/* human-readable plan (layers, fused epilogues, flat buffer, buckets); returns the length */
int64_t fmn_model_describe(fmn_model_t m, char* buf, int64_t len);

#ifdef __cplusplus
}
#endif
#endif /* FLEXMI_NATIVE_C_H */
