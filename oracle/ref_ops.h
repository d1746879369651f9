/* ORACLE — test infrastructure only (see ref_ops.c header). */
#ifndef OREF_OPS_H
#define OREF_OPS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

float oref_ndarray_sum(const float* xs, int64_t n);
int oref_same_padding(int64_t in_h, int64_t in_w, int64_t sh, int64_t sw, int64_t kh, int64_t kw,
                      int64_t pads_tlbr[4]);
int oref_resolve_window(int auto_pad, const int64_t* pads_attr, int n_pads, int64_t H, int64_t W,
                        int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t pads_tlbr[4],
                        int64_t* Ho, int64_t* Wo);
int oref_conv2d(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, const float* w, int64_t M,
                int64_t kh, int64_t kw, const float* bias, const int64_t pads_tlbr[4], int64_t sh,
                int64_t sw, int64_t Ho, int64_t Wo, float* y, int faithful);
int oref_maxpool2d(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, int64_t kh, int64_t kw,
                   const int64_t pads_tlbr[4], int64_t sh, int64_t sw, int64_t Ho, int64_t Wo,
                   float* y, int faithful);
void oref_relu(const float* x, int64_t n, float* y);
int oref_add_bcast(const float* a, const int64_t* adims, int ra, const float* b, const int64_t* bdims,
                   int rb, float* y);
void oref_softmax_rows(const float* x, int64_t rows, int64_t D, float* y);
void oref_matmul(const float* a, const float* b, int64_t M, int64_t K, int64_t Ncols, float* y);
void oref_gap(const float* x, int64_t N, int64_t C, int64_t HW, float* y);
int oref_concat2(const float* a, const int64_t* ad, const float* b, const int64_t* bd, int axis,
                 float* y);

/* Whole-model restatement of inference()/node_inference() (model_inference.rs:29-162). */
typedef struct oref_model oref_model;
oref_model* oref_model_load(const uint8_t* bytes, int64_t len);
void oref_model_free(oref_model* m);
/* Runs the graph in file order on a batch of n images of the model's input shape.
 * out receives graph.output[0] (n * out_elems floats).  Returns 0, or -1 with oref_last_error. */
int oref_model_run(oref_model* m, const float* input, int64_t n, float* out, int64_t out_cap,
                   int faithful);
int64_t oref_model_out_elems(oref_model* m); /* per image, after a successful run */
const char* oref_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
