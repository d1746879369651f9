/*
 * ore.h — C ABI of the MI355X-native (gfx950) fp32 ONNX op executor.
 *
 * Drop-in boundary for the fp32 op path of jackperlo/onnx-rusty-inference-engine.  The
 * reference dispatches every node through `node_inference`
 * (src/inference_engine/model_inference.rs:128-162, match at :137-161) into one Rust function
 * per op in src/inference_fp32_ops/.  Each entry point below replaces one of those functions
 * (cited on the declaration), operating on device tensors that stay resident in HBM.  The
 * graph-level entry points (ore_model_*) replace `inference()` (model_inference.rs:29-120)
 * together with the tensor plumbing of src/inference_engine/utils.rs.
 *
 * Conventions
 *  - Every function returns an ore_status (0 = ORE_OK).  Nothing throws or aborts across the
 *    ABI; the message of the last failure on a context is ore_last_error(ctx) (or
 *    ore_last_error(NULL) for failures before a context exists).  The reference panics in the
 *    same situations (unknown op / attribute / auto_pad string, missing input, shape mismatch).
 *  - Tensors are fp32, NCHW row-major, device memory.  `nstride` is the element distance
 *    between consecutive images (0 = contiguous); it lets an op write a channel slice of a
 *    wider tensor (Concat in place).
 *  - Launches are asynchronous on the context's HIP stream; ore_sync() joins.  A context is
 *    bound to one device and is not thread-safe (one per host thread / device).
 *  - Padding is resolved exactly as the reference does (including its SAME split with the
 *    larger half at the top/left, convolution_op.rs:519-557) before any kernel is launched.
 */
#ifndef ORE_H
#define ORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 2 (round 4) against ABI 1: the opt-in bf16x3 kernels are gone -- load flags 2 / 8 (ABI 1's
 * ORE_LOAD_X3 / ORE_LOAD_X3_ALL) and conv tile ids 28-35 are rejected with ORE_ERR_UNSUPPORTED; so are
 * ABI 1's retired fusion bit 16 (ORE_FUSE_POOL_CONV), MaxPool variant 1 and conv tile ids 4-11, which
 * ABI 1 builds already refused.  ore_model_load accepts any max_batch: a batch whose activations
 * would pass the kernels' 32-bit offsets runs in image chunks inside ore_model_run.  Every other
 * entry point and value is unchanged. */
#define ORE_ABI_VERSION 2

typedef enum ore_status {
  ORE_OK = 0,
  ORE_ERR_INVALID = 1,     /* bad argument / shape mismatch (reference: assert / unwrap panic) */
  ORE_ERR_UNSUPPORTED = 2, /* op, attribute or mode the reference does not implement (panic!) */
  ORE_ERR_HIP = 3,         /* HIP runtime failure */
  ORE_ERR_OOM = 4,         /* device allocation failed */
  ORE_ERR_PARSE = 5        /* malformed ONNX protobuf */
} ore_status;

typedef enum ore_auto_pad {
  ORE_PAD_NOTSET = 0,     /* explicit `pads` */
  ORE_PAD_SAME_UPPER = 1,
  ORE_PAD_SAME_LOWER = 2,
  ORE_PAD_VALID = 3
} ore_auto_pad;

typedef struct ore_ctx ore_ctx;
typedef struct ore_model ore_model;

typedef struct ore_tensor {
  float* data;      /* device pointer to element [0,0,0,0] */
  int32_t ndim;     /* 1..4 */
  int64_t dims[4];
  int64_t nstride;  /* elements between images (dims[0] steps); 0 = contiguous */
} ore_tensor;

/* Conv attributes (convolution_op.rs:132-173).  pads use ONNX order
 * [h_begin, w_begin, h_end, w_end]; n_pads = 0 when the attribute is absent.  As in the
 * reference, any positive pad forces NOTSET (:169-173) and kernel_shape is ignored (:151). */
typedef struct ore_conv_attrs {
  int32_t auto_pad;      /* ore_auto_pad; reference default VALID (:134) */
  int32_t n_pads;
  int64_t pads[4];
  int64_t strides[2];    /* required (the reference unwraps them, :285-290) */
  int64_t dilations[2];  /* must be 1 (dilation > 1 is not a working path in the reference) */
  int64_t group;         /* must be 1 (asserted, :252) */
  int32_t fuse_relu;     /* extension: apply Relu in the epilogue (a following Relu node) */
} ore_conv_attrs;

/* MaxPool attributes (max_pool_op.rs:85-114).  Unlike Conv, pads do NOT force NOTSET: with
 * the default auto_pad (VALID) the pads are ignored, as in the reference. */
typedef struct ore_pool_attrs {
  int32_t auto_pad;
  int32_t n_pads;
  int64_t pads[4];
  int64_t kernel[2];
  int64_t strides[2];
} ore_pool_attrs;

/* ------------------------------------------------------------------ context & memory */
int32_t ore_abi_version(void);
ore_status ore_ctx_create(int32_t device, ore_ctx** out);
ore_status ore_ctx_destroy(ore_ctx* ctx);
/* Launch on an external HIP stream (e.g. the caller's framework stream).  NULL selects the
 * legacy default (null) stream; the context starts on a stream of its own. */
ore_status ore_ctx_set_stream(ore_ctx* ctx, void* hip_stream);
void* ore_ctx_get_stream(ore_ctx* ctx);
ore_status ore_sync(ore_ctx* ctx);
const char* ore_last_error(ore_ctx* ctx);
/* Conv algorithm of the per-op entry ore_conv2d_f32 on this context (extension; the reference has
 * one algorithm, im2col + per-channel dots, convolution_op.rs:224-517).  ORE_CONV_ALGO_DIRECT (the
 * default): the implicit GEMM in the reference's k order.  ORE_CONV_ALGO_WINOGRAD: 3x3 / stride-1 /
 * pad-1 convs with C % 16 == 0 by Winograd F(2x2, 3x3) in f32 (2.25x fewer MFMAs; its error against a
 * float64 reference is at or below the direct f32 conv's, but results are not bit-identical to it);
 * other geometries stay direct.  Models choose per ORE_LOAD_NO_WINOGRAD instead. */
#define ORE_CONV_ALGO_DIRECT 0
#define ORE_CONV_ALGO_WINOGRAD 1
ore_status ore_ctx_set_conv_algo(ore_ctx* ctx, int32_t algo);
/* Kernel selection for parity tests and tuning (extension).  Results never depend on it: every conv
 * tile of one algorithm computes each output by the same k-ordered chain, every MaxPool kernel the
 * same max.
 *  ore_ctx_set_conv_tile: every conv planned on this context afterwards -- ore_conv2d_f32 /
 *    ore_matmul_f32 calls, and models loaded later -- uses tile id `tile` where it belongs to the
 *    layer's kernel family (else the per-layer heuristic); -1 (default) = the heuristic.  Ids as
 *    ore_model_step_tile reports them (0-3 LDS-staged, 12-20 streaming, 36-40 Winograd, 46-48
 *    persistent streaming 1x1); the retired ids 4-11 and 28-35 return ORE_ERR_UNSUPPORTED.
 *  ore_ctx_set_pool_variant: MaxPool kernel of ore_maxpool2d_f32 and of the walker's MaxPool steps:
 *    0 (default) = by layout, 2 one thread per output, 3 column strips, 4 plane-staged, 5
 *    chunk-staged (1 is retired: ORE_ERR_UNSUPPORTED). */
ore_status ore_ctx_set_conv_tile(ore_ctx* ctx, int32_t tile);
ore_status ore_ctx_set_pool_variant(ore_ctx* ctx, int32_t variant);

ore_status ore_malloc(ore_ctx* ctx, size_t bytes, void** dptr);
ore_status ore_free(ore_ctx* ctx, void* dptr);
ore_status ore_upload(ore_ctx* ctx, void* dst, const void* src, size_t bytes);
ore_status ore_download(ore_ctx* ctx, void* dst, const void* src, size_t bytes);

/* ------------------------------------------------------------------ shape inference
 * Output geometry exactly as the reference computes it (convolution_op.rs:292-324,
 * max_pool_op.rs:214-246); pads_tlbr receives the resolved [top, left, bottom, right]. */
ore_status ore_conv_out_shape(const int64_t x_dims[4], const int64_t w_dims[4], const ore_conv_attrs* a,
                              int64_t y_dims[4], int64_t pads_tlbr[4]);
ore_status ore_pool_out_shape(const int64_t x_dims[4], const ore_pool_attrs* a, int64_t y_dims[4],
                              int64_t pads_tlbr[4]);

/* ------------------------------------------------------------------ ops (node_inference arms) */
/* "Conv"     convolution()  convolution_op.rs:94-193 (conv2d :224-517).  x [N,C,H,W],
 *            w [M,C,kh,kw] (ONNX layout), bias [M] or NULL, y [N,M,Ho,Wo] (may be a slice). */
ore_status ore_conv2d_f32(ore_ctx* ctx, const ore_tensor* x, const ore_tensor* w, const ore_tensor* bias,
                          const ore_conv_attrs* a, ore_tensor* y);
/* "MaxPool"  max_pool()  max_pool_op.rs:65-129 (max_pool2d :157-360). */
ore_status ore_maxpool2d_f32(ore_ctx* ctx, const ore_tensor* x, const ore_pool_attrs* a, ore_tensor* y);
/* "Relu"     relu()  relu_op.rs:11-29 (relu_wrapper :31-33).  y may alias x. */
ore_status ore_relu_f32(ore_ctx* ctx, const ore_tensor* x, ore_tensor* y);
/* "Add"      add()  add_op.rs:16-107: a + b with b broadcast right-aligned onto a
 *            ([N,C,H,W] + [C,1,1], or [N,K] + [1,K]). */
ore_status ore_add_f32(ore_ctx* ctx, const ore_tensor* a, const ore_tensor* b, ore_tensor* y);
/* "Softmax"  softmax()  softmax_op.rs:13-42 (softmax_wrapper :45-57): rows = dims[0],
 *            row length = product of the remaining dims; y is [rows, D]. */
ore_status ore_softmax_f32(ore_ctx* ctx, const ore_tensor* x, ore_tensor* y);
/* "MatMul"   mul()  mul_op.rs:11-32: y[M,N] = a[M,K] . b[K,N] (MFMA). */
ore_status ore_matmul_f32(ore_ctx* ctx, const ore_tensor* a, const ore_tensor* b, ore_tensor* y);
/* "GlobalAveragePool"  global_average_pool()  global_average_pool_op.rs:11-51: y [N,C,1,1]. */
ore_status ore_gap_f32(ore_ctx* ctx, const ore_tensor* x, ore_tensor* y);
/* "Concat"   concatenation()  concatenate_op.rs:11-41: exactly two inputs on `axis`. */
ore_status ore_concat_f32(ore_ctx* ctx, const ore_tensor* a, const ore_tensor* b, int64_t axis, ore_tensor* y);
/* "Dropout"  drop_out()  dropout_op.rs:12-89: inference identity (training_mode = false).
 *            Copies when y != x, no-op when they alias. */
ore_status ore_dropout_f32(ore_ctx* ctx, const ore_tensor* x, ore_tensor* y);
/* "Reshape"  reshape()  reshape_op.rs:16-92: metadata only (row-major reinterpretation to
 *            2-D; a 0 in `shape` copies the input dim).  Writes the resulting view to y. */
ore_status ore_reshape(const ore_tensor* x, const int64_t* shape, int32_t n_shape, ore_tensor* y);

/* ------------------------------------------------------------------ graph walker (inference()) */
/* Parse an ONNX ModelProto (bytes), upload every initializer to HBM once, plan the value
 * buffers for up to max_batch images, and prepare the node list in file order.  Any max_batch is
 * accepted: the arena holds run_batch = min(max_batch, the largest batch whose every activation fits
 * the kernels' 32-bit byte offsets) images (ore_model_run_batch), and larger runs go in image chunks.
 * Unsupported ops/attributes fail here (the reference panics when it reaches them). */
ore_status ore_model_load(ore_ctx* ctx, const void* onnx_bytes, size_t len, int64_t max_batch,
                          ore_model** out);
/* Host-only wire-format check of an ONNX ModelProto, the reference's
 * `ModelProto::parse_from_bytes` (main.rs:30) before any inference: ORE_OK, or ORE_ERR_PARSE for
 * malformed protobuf (truncated payloads, a field sent with the wrong wire type, ...) with the
 * reason in ore_last_error(NULL).  Touches no device; ore_model_load runs the same parser. */
ore_status ore_model_parse(const void* onnx_bytes, size_t len);
/* Load flags.  ORE_LOAD_F16: the fp16 variant (no reference
 * counterpart -- the reference is f32 only): Conv weights and the activations of Conv / MaxPool /
 * Relu / Concat / Dropout are f16, Conv accumulates in f32 on the f16 matrix cores (bias and Relu
 * in f32, rounded once), GlobalAveragePool sums f16 inputs in f32, and Softmax, Add and MatMul
 * stay f32 (Add / MatMul / Softmax on an f16 value is rejected).  The model input and
 * graph.output[0] stay f32 (an f16 graph output is rejected). */
#define ORE_LOAD_F16 1
/* ORE_LOAD_NO_WINOGRAD: an f32 model runs its 3x3 / stride-1 / pad-1 convs (SqueezeNet's
 * expand3x3) on the direct kernels only, every output in the reference's k order.  By default (f32
 * models) every such conv with C % 16 == 0 that no direct-kernel fusion takes runs Winograd
 * F(2x2, 3x3) in f32 (ore_conv_wino.hip; see ORE_CONV_ALGO_WINOGRAD above).  NOTE: this makes the
 * default f32 results differ from the direct path by rounding (synthetic SqueezeNet @224: 6e-6
 * max-abs against the oracle vs 2e-7 direct, within the 1e-5 parity bound); load with this flag for
 * the reference's summation order.  The choice is made at load time, never by timing. */
#define ORE_LOAD_NO_WINOGRAD 4
/* ABI 1's ORE_LOAD_X3 (2) and ORE_LOAD_X3_ALL (8): retired, rejected with ORE_ERR_UNSUPPORTED. */
#define ORE_LOAD_RETIRED_MASK 10
ore_status ore_model_load_ex(ore_ctx* ctx, const void* onnx_bytes, size_t len, int64_t max_batch, int32_t flags,
                             ore_model** out);
ore_status ore_model_destroy(ore_model* m);
/* Fusion flags (ore_model_set_fusion; ORE_FUSE_ALL is the default, 0 runs every node as its own kernel
 * for op-by-op parity).  Every fusion is exact: the fused kernels compute each output by the same
 * arithmetic as the separate ones, so results do not depend on the flags (tested bit for bit).
 * bit 0 = fuse Conv->Relu, bit 1 = Concat in place (and padded channel planes), bit 2 = alias
 * Dropout / Reshape; bits 5-10 and 12 below.  Bit 4 (ABI 1's ORE_FUSE_POOL_CONV, a MaxPool inside a
 * 1x1 conv's operand gather, measured slower) is retired: ORE_ERR_UNSUPPORTED. */
#define ORE_FUSE_CONV_RELU 1
#define ORE_FUSE_CONCAT 2
#define ORE_FUSE_ALIAS 4
#define ORE_FUSE_ALL 14311
/* bit 5 (in ORE_FUSE_ALL): Conv (-> Relu) -> 3x3 / stride-2 MaxPool as ONE launch when the conv
 * output has no other consumer: each block computes a 13 x 19 patch of conv outputs covering a
 * 6 x 9 tile of pooled outputs (the overlapping window row / column is recomputed by the
 * neighbouring tile) and stores only the pooled values; the pre-pool tensor never reaches HBM.
 * Bit-identical (same per-output MFMA chain; max is exact).  Applied when the computed columns are
 * <= 1.25 x the conv's own (SqueezeNet @224: conv1 + pool1 only, 1.16x).  f32 models: ore_model_autotune also times the row-walking kernels
 * (ore_conv_pool.hip: a block walks the conv plane row-major and max-reduces into an LDS ring of
 * pooled rows, nothing recomputed) and keeps the fastest -- conv1 + pool1: 96 channels x 128
 * quads per block, 1016 -> ~900 us at batch 256. */
#define ORE_FUSE_CONV_POOL 32
/* bit 6: a fire module (Concat of a 1x1 and a 3x3 'same' Conv + Relu of one value, 64-multiple
 * channel counts) and the 1x1 Conv + Relu (<= 64 channels) that is the Concat's only reader -- the
 * next fire's squeeze -- as ONE launch: the expand outputs and the Concat never reach HBM.
 * Bit-identical (every output keeps its k-ordered MFMA chain; the squeeze still sums the concat
 * channels in ascending order).  f32 (fire_kernel) and f16 (fire_f16_kernel) models; f32: applied when
 * max_batch * H * W >= 65536 (one 64-pixel wave per SIMD), below which the fused launch has too few
 * waves (batch 1 keeps the separate kernels).  f16 models also take a fire module whose Concat is
 * read by something other than a squeeze (SqueezeNet's fire9, read by conv10): its expands and the
 * Concat run as one fire_f16_kernel launch that stores the Concat. */
#define ORE_FUSE_FIRE 64
/* bit 7 (in ORE_FUSE_ALL): Concat(e1, e3) -> 3x3 / stride-2 MaxPool with e1 / e3 Convs
 * (+ Relu) read only by the Concat (SqueezeNet's fire4 -> pool3, fire8 -> pool5): each conv's pooled
 * epilogue (the row-walking kernel, ore_conv_pool.hip) writes its channel slice of the pool output,
 * so neither the expand outputs nor the Concat reach HBM.  Bit-identical (the pool is per channel;
 * every pooled value is the max of the same nine values).  f32 models, conv planes of at least 1024
 * pixels: at batch 256 fire4 -> pool3 (54 x 54) saves 40 us per step, fire8 -> pool5 (27 x 27)
 * would cost 21 us (the walker's expand3x3 runs at 88-92 % of the streaming kernel's rate). */
#define ORE_FUSE_CONCAT_POOL 128
/* bit 8: a fire module, the 3x3 / stride-2 MaxPool of its Concat and the next squeeze as ONE launch
 * (f32 fire_pool_kernel on expand planes of >= 1024 pixels at max_batch * H * W >= 65536: fire4 +
 * pool3 + fire5/squeeze; f16 fire_pool_f16_kernel: also fire8 + pool5 + fire9/squeeze). */
#define ORE_FUSE_FIRE_POOL 256
/* bit 9: the first conv + its pooled epilogue also runs the pooled map's only reader, a 1x1 conv
 * (+ Relu) with <= 16 (f32) / 32 (f16) channels (conv1 + pool1 + fire2/squeeze). */
#define ORE_FUSE_FIRST_SQUEEZE 512
/* bit 10: a 3x3 / stride-2 MaxPool read only by a 1x1 conv (+ Relu, <= 64 channels) runs inside that
 * conv (f32 pool_conv1x1_f32_kernel: pool5 + fire9/squeeze). */
#define ORE_FUSE_POOL_SQUEEZE 1024
/* bit 12: a 1x1 conv (+ Relu) whose only reader is GlobalAveragePool runs with the GAP in its
 * epilogue: conv10 + relu10 + pool10 in one launch, the conv map never stored (f16 models:
 * conv1x1_gap_f16_kernel; f32 models since round 4: conv1x1_gap_f32_kernel, input channels a multiple
 * of 32, <= 256 pixels).  Bit-identical to the separate launches; not under ORE_KEEP_VALUES. */
#define ORE_FUSE_CONV_GAP 4096
/* bit 13 (round 5): with ORE_FUSE_POOL_SQUEEZE, a pool whose input is Concat(e1, e3) with e1 a 1x1
 * conv (+ Relu) of 32 / 64 channels read only by the Concat: e1 is recomputed inside the pooled
 * squeeze from its own input, so its map is never stored (SqueezeNet fire4 -> pool3 -> fire5 and
 * fire8 -> pool5 -> fire9 when their expand3x3 runs Winograd).  Bit-identical; f32 models; not
 * under ORE_KEEP_VALUES. */
#define ORE_FUSE_POOL_EXPAND 8192
/* bit 11 (tests, not in ORE_FUSE_ALL): apply every eligible fusion regardless of the size
 * heuristics above (batch / plane thresholds, the 1.25 patch-work bound). */
#define ORE_FUSE_EAGER 2048
/* debug: give every value its own storage (no liveness reuse) so any value can be read back */
#define ORE_KEEP_VALUES 8
ore_status ore_model_set_fusion(ore_model* m, int32_t flags);
/* The seeded model input (graph.input entries that are not initializers, utils.rs:29-45):
 * per-image dims; dims[0] is the batch. */
ore_status ore_model_input_dims(ore_model* m, int64_t dims[4]);
/* Elements per image of graph.output[0] (the reference only prints it; we keep it). */
ore_status ore_model_output_elems(ore_model* m, int64_t* elems);
/* Run all nodes on n <= max_batch images.  d_input/d_output are device pointers
 * (n * input elems / n * output elems).  Asynchronous on the context stream.  n > run_batch runs the
 * graph once per chunk of at most run_batch consecutive images (each image's arithmetic is the same
 * in any chunk). */
ore_status ore_model_run(ore_model* m, const float* d_input, int64_t n, float* d_output);
/* Images one pass of the graph covers (see ore_model_load). */
int64_t ore_model_run_batch(ore_model* m);
/* Copy a named value of the last run to host memory (for node-level parity checks; values
 * elided by fusion, and values of a run chunked over run_batch, are unavailable -> ORE_ERR_INVALID).
 * Synchronises. */
ore_status ore_model_read_value(ore_model* m, const char* name, float* host_dst, size_t cap_elems,
                                int64_t dims[4], int32_t* ndim);
/* Per-node timing with HIP events on the context stream (enable, run, then query).
 * ore_model_node_count/ore_model_node_info describe the executed kernel steps. */
/* Measure every Conv step's candidate block tiles (128x128, 96x128, 64x128, 32x256) on a real
 * run of n images (d_input / d_output as for ore_model_run) and keep the fastest per layer (like
 * a benchmark-mode convolution search).  Results do not depend on the tile.  Synchronous.
 * reps: timed launches per candidate (<= 0: 3).  The choice survives ore_model_set_fusion.  A batch
 * above run_batch is tuned on its first chunk, then run whole once, so on return d_output holds the
 * output of all n images either way. */
ore_status ore_model_autotune(ore_model* m, const float* d_input, int64_t n, float* d_output, int32_t reps);
/* Block tile chosen for exec step i (-1 for non-conv steps); steps with one fixed kernel report its
 * id (e.g. 49 / 50: conv + GlobalAveragePool, f16 / f32).  The f32 first conv + pool + squeeze step
 * has two: 44 (13 x 19 patches) and 51 (the band walker, round 5); the f16 one 43 (patches) and 52 (the
 * f16 band walker, round 6).  The autotune keeps the faster. */
int32_t ore_model_step_tile(ore_model* m, int32_t i);
/* Set exec step i's tile (one of the ids ore_model_autotune chooses among for that step; e.g. to
 * restore a saved autotune result).  ORE_ERR_INVALID for an id outside the step's kernel family.
 * Survives ore_model_set_fusion like the autotuned choice. */
ore_status ore_model_set_step_tile(ore_model* m, int32_t i, int32_t tile);
/* MFMA FLOPs exec step i issued in the last run: its algorithmic FLOPs (ore_model_step_info), except
 * Winograd steps, which issue 16 C M per 2x2 output tile against the direct 36 C M. */
ore_status ore_model_step_mfma_flops(ore_model* m, int32_t i, double* flops);
/* Branch concurrency (the reference runs the two expand branches of a fire
 * module on threads, multithreading.rs:20-62): with 2 streams, adjacent independent steps (no
 * data dependence, no overlapping storage) run on a side stream beside the main one, joined by
 * events.  Pays off at small batch, where one conv does not fill the GPU.  Default 1. */
ore_status ore_model_set_streams(ore_model* m, int32_t streams);
/* Capture one ore_model_run(d_input, n, d_output) into a HIP graph (launch-bound small batches:
 * one graph launch replaces ~30 kernel launches); replay it with ore_model_graph_launch on the
 * context stream.  The graph keeps the buffers and batch it was captured with; re-capture after
 * ore_model_set_fusion / set_streams.  Needs a non-null context stream. */
ore_status ore_model_graph_capture(ore_model* m, const float* d_input, int64_t n, float* d_output);
ore_status ore_model_graph_launch(ore_model* m);
ore_status ore_model_enable_timing(ore_model* m, int32_t on);
int32_t ore_model_step_count(ore_model* m);
ore_status ore_model_step_info(ore_model* m, int32_t i, const char** op, const char** name, double* flops,
                               double* bytes);
ore_status ore_model_step_times(ore_model* m, float* ms, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* ORE_H */
