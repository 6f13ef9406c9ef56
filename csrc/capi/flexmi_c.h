/* flexmi C API -- the CPython-EMBEDDING model API (C-API parity with the reference's
 * python/flexflow_c.h:49-749).  For C programs that must not load Python at all, use the native
 * API in flexmi_native_c.h (libflexmi_native_c.so: the C++ runtime, plan compiler for DLRM and
 * CNN graphs, simulator / search, loaders -- no interpreter).
 *
 * Opaque handles over the flexmi runtime.  The library embeds CPython when the host program is
 * not Python (a C/C++ application calls flexmi_init first) and works from inside a Python
 * process too (ctypes).  Every function returns NULL / a negative value on error; the message
 * is available from flexmi_last_error().
 *
 * Dimension order is the natural (row-major, batch-first) order of the Python API: a dense
 * input is {batch, features}, an image {batch, channels, height, width}.  Enum values are the
 * reference's (include/ffconst.h): ActiMode NONE=10 RELU=11 SIGMOID=12 TANH=13; AggrMode
 * NONE=20 SUM=21 AVG=22; PoolType MAX=30 AVG=31; DataType FLOAT=40 DOUBLE=41 INT32=42 INT64=43;
 * LossType CCE=50 SPARSE_CCE=51 MSE_AVG=52 MSE_SUM=53; Metrics ACCURACY=1001 CCE=1002
 * SPARSE_CCE=1004 MSE=1008 RMSE=1016 MAE=1032.
 */
#ifndef FLEXMI_C_H
#define FLEXMI_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLEXMI_HANDLE(name) typedef struct name##_s* name##_t
FLEXMI_HANDLE(flexmi_config);
FLEXMI_HANDLE(flexmi_model);
FLEXMI_HANDLE(flexmi_tensor);
FLEXMI_HANDLE(flexmi_parameter);
FLEXMI_HANDLE(flexmi_op);
FLEXMI_HANDLE(flexmi_optimizer);
FLEXMI_HANDLE(flexmi_initializer);
FLEXMI_HANDLE(flexmi_perf_metrics);
FLEXMI_HANDLE(flexmi_dataloader);
#undef FLEXMI_HANDLE

/* ---- runtime ---------------------------------------------------------------------------- */
int flexmi_init(int argc, char** argv); /* idempotent; argv becomes sys.argv (flag parsing) */
void flexmi_finalize(void);
const char* flexmi_last_error(void);
double flexmi_get_current_time(flexmi_config_t config); /* microseconds */
void flexmi_begin_trace(flexmi_config_t config, int trace_id);
void flexmi_end_trace(flexmi_config_t config, int trace_id);

/* ---- config ------------------------------------------------------------------------------ */
flexmi_config_t flexmi_config_create(void);
void flexmi_config_destroy(flexmi_config_t c);
int flexmi_config_parse_args(flexmi_config_t c, int argc, char** argv);
int flexmi_config_parse_args_default(flexmi_config_t c); /* from flexmi_init's argv */
int flexmi_config_get_batch_size(flexmi_config_t c);
int flexmi_config_set_batch_size(flexmi_config_t c, int batch);
int flexmi_config_get_workers_per_node(flexmi_config_t c);
int flexmi_config_get_num_nodes(flexmi_config_t c);
int flexmi_config_get_epochs(flexmi_config_t c);
int flexmi_config_set_device(flexmi_config_t c, const char* device); /* "cpu" | "gpu" */

/* ---- model lifecycle ---------------------------------------------------------------------- */
flexmi_model_t flexmi_model_create(flexmi_config_t c);
void flexmi_model_destroy(flexmi_model_t m);
int flexmi_model_compile(flexmi_model_t m, flexmi_optimizer_t opt, int loss_type, const int* metrics, int n_metrics);
int flexmi_model_init_layers(flexmi_model_t m);
int flexmi_model_forward(flexmi_model_t m);
int flexmi_model_backward(flexmi_model_t m);
int flexmi_model_update(flexmi_model_t m);
int flexmi_model_zero_gradients(flexmi_model_t m);
int flexmi_model_reset_metrics(flexmi_model_t m);
int flexmi_model_compute_metrics(flexmi_model_t m);
int flexmi_model_prefetch(flexmi_model_t m);
int flexmi_model_print_layers(flexmi_model_t m, int id);
int flexmi_model_set_sgd_optimizer(flexmi_model_t m, flexmi_optimizer_t opt);
int flexmi_model_set_adam_optimizer(flexmi_model_t m, flexmi_optimizer_t opt);
flexmi_tensor_t flexmi_model_get_label_tensor(flexmi_model_t m);
flexmi_op_t flexmi_model_get_layer_by_id(flexmi_model_t m, int id);
flexmi_parameter_t flexmi_model_get_parameter_by_id(flexmi_model_t m, int id);
flexmi_perf_metrics_t flexmi_model_get_perf_metrics(flexmi_model_t m);
int flexmi_model_save_checkpoint(flexmi_model_t m, const char* path);
int flexmi_model_load_checkpoint(flexmi_model_t m, const char* path);

/* ---- builders (return the output tensor) ------------------------------------------------- */
flexmi_tensor_t flexmi_tensor_create(flexmi_model_t m, int ndims, const int* dims, int data_type, int create_grad,
                                     const char* name);
flexmi_tensor_t flexmi_model_add_exp(flexmi_model_t m, flexmi_tensor_t x, const char* name);
flexmi_tensor_t flexmi_model_add_relu(flexmi_model_t m, flexmi_tensor_t x, const char* name);
flexmi_tensor_t flexmi_model_add_sigmoid(flexmi_model_t m, flexmi_tensor_t x, const char* name);
flexmi_tensor_t flexmi_model_add_tanh(flexmi_model_t m, flexmi_tensor_t x, const char* name);
flexmi_tensor_t flexmi_model_add_elu(flexmi_model_t m, flexmi_tensor_t x, const char* name);
flexmi_tensor_t flexmi_model_add_add(flexmi_model_t m, flexmi_tensor_t x, flexmi_tensor_t y, const char* name);
flexmi_tensor_t flexmi_model_add_subtract(flexmi_model_t m, flexmi_tensor_t x, flexmi_tensor_t y, const char* name);
flexmi_tensor_t flexmi_model_add_multiply(flexmi_model_t m, flexmi_tensor_t x, flexmi_tensor_t y, const char* name);
flexmi_tensor_t flexmi_model_add_divide(flexmi_model_t m, flexmi_tensor_t x, flexmi_tensor_t y, const char* name);
flexmi_tensor_t flexmi_model_add_conv2d(flexmi_model_t m, flexmi_tensor_t x, int out_channels, int kernel_h,
                                        int kernel_w, int stride_h, int stride_w, int padding_h, int padding_w,
                                        int activation, int use_bias, flexmi_initializer_t kernel_init,
                                        flexmi_initializer_t bias_init, const char* name);
flexmi_tensor_t flexmi_model_add_embedding(flexmi_model_t m, flexmi_tensor_t x, int num_entries, int out_dim,
                                           int aggr, flexmi_initializer_t kernel_init, const char* name);
flexmi_tensor_t flexmi_model_add_pool2d(flexmi_model_t m, flexmi_tensor_t x, int kernel_h, int kernel_w, int stride_h,
                                        int stride_w, int padding_h, int padding_w, int pool_type, int activation,
                                        const char* name);
flexmi_tensor_t flexmi_model_add_batch_norm(flexmi_model_t m, flexmi_tensor_t x, int relu, const char* name);
flexmi_tensor_t flexmi_model_add_batch_matmul(flexmi_model_t m, flexmi_tensor_t a, flexmi_tensor_t b,
                                              const char* name);
flexmi_tensor_t flexmi_model_add_dense(flexmi_model_t m, flexmi_tensor_t x, int out_dim, int activation,
                                       int use_bias, flexmi_initializer_t kernel_init, flexmi_initializer_t bias_init,
                                       const char* name);
flexmi_tensor_t flexmi_model_add_concat(flexmi_model_t m, int n, const flexmi_tensor_t* xs, int axis,
                                        const char* name);
/* outputs: caller array of n handles */
int flexmi_model_add_split(flexmi_model_t m, flexmi_tensor_t x, int n, const int* sizes, int axis,
                           flexmi_tensor_t* outputs, const char* name);
flexmi_tensor_t flexmi_model_add_flat(flexmi_model_t m, flexmi_tensor_t x, const char* name);
flexmi_tensor_t flexmi_model_add_softmax(flexmi_model_t m, flexmi_tensor_t x, const char* name);
flexmi_tensor_t flexmi_model_add_reshape(flexmi_model_t m, flexmi_tensor_t x, int ndims, const int* shape,
                                         const char* name);
flexmi_tensor_t flexmi_model_add_transpose(flexmi_model_t m, flexmi_tensor_t x, int ndims, const int* perm,
                                           const char* name);
flexmi_tensor_t flexmi_model_add_reverse(flexmi_model_t m, flexmi_tensor_t x, int axis, const char* name);
flexmi_tensor_t flexmi_model_add_dropout(flexmi_model_t m, flexmi_tensor_t x, float rate, unsigned long long seed,
                                         const char* name);

/* ---- tensors / parameters / ops ----------------------------------------------------------- */
void flexmi_tensor_destroy(flexmi_tensor_t t);
int flexmi_tensor_get_num_dims(flexmi_tensor_t t);
int flexmi_tensor_get_dims(flexmi_tensor_t t, int* dims); /* returns ndims */
int flexmi_tensor_get_data_type(flexmi_tensor_t t);
flexmi_op_t flexmi_tensor_get_owner_op(flexmi_tensor_t t);
/* whole logical tensor <-> host buffer (inline_map + copy + inline_unmap) */
int flexmi_tensor_set_array_float(flexmi_model_t m, flexmi_tensor_t t, const float* data, size_t n);
int flexmi_tensor_get_array_float(flexmi_model_t m, flexmi_tensor_t t, float* out, size_t n);
int flexmi_tensor_set_array_int32(flexmi_model_t m, flexmi_tensor_t t, const int32_t* data, size_t n);
int flexmi_tensor_set_array_int64(flexmi_model_t m, flexmi_tensor_t t, const int64_t* data, size_t n);
void flexmi_parameter_destroy(flexmi_parameter_t p);
int flexmi_parameter_get_num_elements(flexmi_parameter_t p);
int flexmi_parameter_get_weights_float(flexmi_parameter_t p, flexmi_model_t m, float* out, size_t n);
int flexmi_parameter_set_weights_float(flexmi_parameter_t p, flexmi_model_t m, const float* data, size_t n);
void flexmi_op_destroy(flexmi_op_t op);
flexmi_parameter_t flexmi_op_get_parameter_by_id(flexmi_op_t op, int id);
flexmi_tensor_t flexmi_op_get_input_by_id(flexmi_op_t op, int id);
flexmi_tensor_t flexmi_op_get_output_by_id(flexmi_op_t op, int id);
int flexmi_op_get_name(flexmi_op_t op, char* buf, size_t len);

/* ---- optimizers / initializers / metrics -------------------------------------------------- */
flexmi_optimizer_t flexmi_sgd_optimizer_create(flexmi_model_t m, double lr, double momentum, int nesterov,
                                               double weight_decay);
flexmi_optimizer_t flexmi_adam_optimizer_create(flexmi_model_t m, double alpha, double beta1, double beta2,
                                                double weight_decay, double epsilon);
int flexmi_optimizer_set_lr(flexmi_optimizer_t o, double lr);
void flexmi_optimizer_destroy(flexmi_optimizer_t o);
flexmi_initializer_t flexmi_glorot_uniform_initializer_create(int seed);
flexmi_initializer_t flexmi_zero_initializer_create(void);
flexmi_initializer_t flexmi_uniform_initializer_create(int seed, float min_val, float max_val);
flexmi_initializer_t flexmi_norm_initializer_create(int seed, float mean, float stddev);
void flexmi_initializer_destroy(flexmi_initializer_t i);
float flexmi_perf_metrics_get_accuracy(flexmi_perf_metrics_t pm);
float flexmi_perf_metrics_get_loss(flexmi_perf_metrics_t pm);
void flexmi_perf_metrics_destroy(flexmi_perf_metrics_t pm);

/* ---- data loaders ------------------------------------------------------------------------- */
/* full dataset [num_samples, tensor dims[1:]...] copied from `data` (data_type as DataType) */
flexmi_dataloader_t flexmi_single_dataloader_create(flexmi_model_t m, flexmi_tensor_t t, const void* data,
                                                    int num_samples, int data_type);
int flexmi_dataloader_next_batch(flexmi_dataloader_t d, flexmi_model_t m);
int flexmi_dataloader_reset(flexmi_dataloader_t d);
int flexmi_dataloader_get_num_samples(flexmi_dataloader_t d);
int flexmi_dataloader_set_num_samples(flexmi_dataloader_t d, int n);
void flexmi_dataloader_destroy(flexmi_dataloader_t d);

/* ---- reference-name parity (python/flexflow_c.h): typed aliases and the remaining entry points */
typedef struct flexmi_net_config_s* flexmi_net_config_t;
typedef flexmi_dataloader_t flexmi_dataloader_2d_t;
typedef flexmi_dataloader_t flexmi_dataloader_4d_t;
typedef flexmi_dataloader_t flexmi_single_dataloader_t;
typedef flexmi_perf_metrics_t flexmi_per_metrics_t;

void flexmi_sgd_optimizer_destroy(flexmi_optimizer_t o);
int flexmi_sgd_optimizer_set_lr(flexmi_optimizer_t o, double lr);
void flexmi_adam_optimizer_destroy(flexmi_optimizer_t o);
int flexmi_adam_optimizer_set_lr(flexmi_optimizer_t o, double lr);
flexmi_initializer_t flexmi_initializer_create_null(void); /* "no initializer": the op's default */
void flexmi_glorot_uniform_initializer_destroy(flexmi_initializer_t i);
void flexmi_zero_initializer_destroy(flexmi_initializer_t i);
void flexmi_uniform_initializer_destroy(flexmi_initializer_t i);
void flexmi_norm_initializer_destroy(flexmi_initializer_t i);
float flexmi_per_metrics_get_accuracy(flexmi_per_metrics_t pm);
void flexmi_per_metrics_destroy(flexmi_per_metrics_t pm);

/* constant tensor (every element = value) */
flexmi_tensor_t flexmi_constant_create(flexmi_model_t m, int num_dims, const int* dims, float value, int data_type);

/* functional ("no in/out") layers: built without an input, connected by flexmi_op_init_inout */
flexmi_op_t flexmi_model_add_conv2d_no_inout(flexmi_model_t m, int in_channels, int out_channels, int kh, int kw, int sh,
                                             int sw, int ph, int pw, int act, int use_bias, flexmi_initializer_t ki,
                                             flexmi_initializer_t bi);
flexmi_op_t flexmi_model_add_pool2d_no_inout(flexmi_model_t m, int kh, int kw, int sh, int sw, int ph, int pw,
                                             int pool_type, int act);
flexmi_op_t flexmi_model_add_dense_no_inout(flexmi_model_t m, int in_dim, int out_dim, int act, int use_bias,
                                            flexmi_initializer_t ki, flexmi_initializer_t bi);
flexmi_op_t flexmi_model_add_flat_no_inout(flexmi_model_t m);
flexmi_tensor_t flexmi_op_init_inout(flexmi_op_t op, flexmi_model_t m, flexmi_tensor_t input);
int flexmi_op_init(flexmi_op_t op, flexmi_model_t m);
/* run this op's forward compute on this rank (its inputs must already be in place) */
int flexmi_op_forward(flexmi_op_t op, flexmi_model_t m);

/* host mapping of a whole logical tensor (config may be NULL) */
int flexmi_tensor_inline_map(flexmi_tensor_t t, flexmi_config_t c);
int flexmi_tensor_inline_unmap(flexmi_tensor_t t, flexmi_config_t c);
int flexmi_tensor_is_mapped(flexmi_tensor_t t);
/* mapped host data (after inline_map), else this rank's device shard */
float* flexmi_tensor_get_raw_ptr_float(flexmi_tensor_t t, flexmi_config_t c);
int32_t* flexmi_tensor_get_raw_ptr_int32(flexmi_tensor_t t, flexmi_config_t c);
/* zero-copy attach of host memory holding the whole logical tensor (column_major: reversed dims) */
int flexmi_tensor_attach_raw_ptr(flexmi_tensor_t t, flexmi_config_t c, void* raw_ptr, int column_major);
int flexmi_tensor_detach_raw_ptr(flexmi_tensor_t t, flexmi_config_t c);

/* NetConfig: --dataset of flexmi_init's argv */
flexmi_net_config_t flexmi_net_config_create(void);
void flexmi_net_config_destroy(flexmi_net_config_t n);
const char* flexmi_net_config_get_dataset_path(flexmi_net_config_t n);

/* input + label loaders.  create: random synthetic data (4 batches) unless the net config names a
 * dataset; create_v2: from host tensors holding the full input / label (attached arrays) */
flexmi_dataloader_4d_t flexmi_dataloader_4d_create(flexmi_model_t m, flexmi_net_config_t n, flexmi_tensor_t input,
                                                   flexmi_tensor_t label);
flexmi_dataloader_4d_t flexmi_dataloader_4d_create_v2(flexmi_model_t m, flexmi_tensor_t input, flexmi_tensor_t label,
                                                      flexmi_tensor_t full_input, flexmi_tensor_t full_label,
                                                      int num_samples);
flexmi_dataloader_2d_t flexmi_dataloader_2d_create_v2(flexmi_model_t m, flexmi_tensor_t input, flexmi_tensor_t label,
                                                      flexmi_tensor_t full_input, flexmi_tensor_t full_label,
                                                      int num_samples);
int flexmi_dataloader_4d_next_batch(flexmi_dataloader_4d_t d, flexmi_model_t m);
int flexmi_dataloader_4d_reset(flexmi_dataloader_4d_t d);
int flexmi_dataloader_4d_get_num_samples(flexmi_dataloader_4d_t d);
int flexmi_dataloader_4d_set_num_samples(flexmi_dataloader_4d_t d, int n);
void flexmi_dataloader_4d_destroy(flexmi_dataloader_4d_t d);
int flexmi_dataloader_2d_next_batch(flexmi_dataloader_2d_t d, flexmi_model_t m);
int flexmi_dataloader_2d_reset(flexmi_dataloader_2d_t d);
int flexmi_dataloader_2d_get_num_samples(flexmi_dataloader_2d_t d);
int flexmi_dataloader_2d_set_num_samples(flexmi_dataloader_2d_t d, int n);
void flexmi_dataloader_2d_destroy(flexmi_dataloader_2d_t d);
int flexmi_single_dataloader_reset(flexmi_single_dataloader_t d);
int flexmi_single_dataloader_get_num_samples(flexmi_single_dataloader_t d);
int flexmi_single_dataloader_set_num_samples(flexmi_single_dataloader_t d, int n);
void flexmi_single_dataloader_destroy(flexmi_single_dataloader_t d);

#ifdef __cplusplus
}
#endif
#endif /* FLEXMI_C_H */
