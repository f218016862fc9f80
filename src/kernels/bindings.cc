// pybind11 bindings for the gfx950 kernels (_hip_kernels.so).
//
// Every entry point takes raw device pointers (as integers), shapes and the
// HIP stream to launch on (torch.cuda.current_stream().cuda_stream), so the
// launches are captured by HIP graphs like any other work on that stream.
// Shape/alignment validation happens in Python (ops/kernel_fns.py) before the
// call; the launchers re-check the invariants they rely on.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace mxamd {
void bn_nhwc_forward(int dtype, const void* x, const void* addend, void* y, uint8_t* mask, const float* gamma,
                     const float* beta,
                     const float* center, float* part, float* mean, float* invstd, float* var, float* scale,
                     float* shift, int64_t R, int C, float eps, int training, int relu, int fix_gamma,
                     float momentum, float* mm_upd, float* mv_upd, int ext_nblk, hipStream_t s);
void bn_nhwc_backward(int dtype, const void* x, const void* dy, const void* y, const uint8_t* mask, void* dx,
                      void* dz,
                      const float* gamma, const float* mean, const float* invstd, const float* fscale,
                      const float* fshift, float* part, float* dgamma, float* dbeta, float* coef, int64_t R, int C,
                      int relu_mode, int fix_gamma, int training, int accum, hipStream_t s, int ext_nblk, const void* ds_z, const float* ds_mean, float* ds_part);
int bn_partials_rows(int64_t R, int C);
int bn_tail_ds_rows(int64_t R, int C);
void gemm_nt(int dtype, const void* a, const void* b, const void* bias, const void* addend, void* c, int out_f32,
             int M, int N, int K, int lda, int ldb, int ldc, int act, int cfg, int splits, float* ws, hipStream_t s,
             int bias_lowp);
int gemm_nt_tile_n(int cfg);
int gemm_nt_tile_m(int cfg);
void int8_gemm(const int8_t* A, const int8_t* B, int32_t* C, int M, int N, int K, hipStream_t s);
void csr_dot_dense(int dtype, const int64_t* indptr, const int64_t* indices, const void* vals, const void* rhs,
                   void* out, int64_t M, int64_t K, int N, hipStream_t s);
void csrT_dot_dense(int dtype, const int64_t* indptr, const int64_t* indices, const void* vals, const void* rhs,
                    const int64_t* slot, float* out32, int64_t M, int64_t K, int N, hipStream_t s);
void embedding_forward(int dtype, int itype, const void* idx, const void* w, void* y, int64_t n, int V, int C,
                       hipStream_t s);
void embedding_backward(int dtype, int itype, const void* idx, const void* dy, float* acc, uint8_t* touched,
                        int out_dtype, void* grad, int accum, int64_t n, int V, int C, hipStream_t s);
int bn_nhwc_stats(int dtype, const void* x, const float* center, float* part, int64_t R, int C, hipStream_t s,
                  int total_blocks);
int64_t colsum_partials(int64_t R, int C);
void colsum_rows(int dtype, const void* x, const float* zeros, float* part, int64_t R, int C, int out_dtype,
                 void* out, int accum, hipStream_t s);
void softmax_ce_forward(int dtype, int label_is_int, const void* logits, const void* label, float* loss, float* lse,
                        int N, int K, hipStream_t s);
void softmax_ce_backward(int dtype, int label_is_int, const void* logits, const void* label, const float* lse,
                         const float* gout, void* dlogits, int N, int K, hipStream_t s);
void gap_nhwc_forward(int dtype, const void* x, void* y, int N, int HW, int C, hipStream_t s);
void relu_forward(int dtype, const void* x, void* y, int64_t n, hipStream_t s);
void relu_backward(int dtype, const void* y, const void* dy, void* dx, int64_t n, hipStream_t s);
void pointwise_binary(int dtype, int op, const void* a, const void* b, void* out, int64_t n, int mode, int64_t row,
                      int ndim, const int64_t* shape, const int64_t* astride, const int64_t* bstride, hipStream_t s);
void gap_nhwc_backward(int dtype, const void* dy, void* dx, int N, int HW, int C, hipStream_t s);
void flat_sgd(int dtype, void* w, const void* g, float* mom, float* w32, int64_t n, float lr, float wd,
              float momentum, float rescale, float clip, const float* hp, hipStream_t s);
void conv_nhwc_fwd(int dtype, const void* x, const void* w, const float* bias, void* y, int N, int H, int W, int C,
                   int K, int R, int S, int sh, int sw, int ph, int pw, int variant, hipStream_t s);
int conv_nhwc_fwd_big_nparts(int N, int H, int W, int R, int S, int sh, int sw, int ph, int pw, int variant);
void conv_nhwc_fwd_big(int dtype, const void* x, const void* w, const float* bias, void* y, const void* zero, int N,
                       int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int variant,
                       float* part, int nparts, const void* addend, hipStream_t s, const void* bn_z,
                       const float* bn_mean, const float* bn_scale, const float* bn_shift, const uint8_t* bn_mask,
                       int bn_mode, float* bn_part, int bn_nparts, int up, int dh, int dw);
int conv_nhwc_fwd_big_bwd_nparts(int N, int H, int W, int R, int S, int sh, int sw, int ph, int pw, int variant);
void conv_nhwc_fwd_glds(int dtype, const void* x, const void* w, const float* bias, void* y, const void* zero, int N,
                        int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int bco,
                        hipStream_t s, const void* bn_z, const float* bn_mean, const float* bn_scale,
                        const float* bn_shift, float* bn_part, int bn_nparts);
int conv_glds_bwd_nparts(int M, int bco);
void conv_nhwc_dgrad_phases_glds(int dtype, const void* dy, const void* w, void* dx, const void* zero, int N, int Hi,
                                 int Wi, int Cin, int Cout, int Ho, int Wo, int stride, int nph, const int* ph,
                                 const int* pw, const int* R, const int* S, const int* pad_h, const int* pad_w,
                                 const int64_t* w_off, int nzero, const int* zph, const int* zpw, int bco,
                                 hipStream_t s, const void* bn_z, const float* bn_mean, const float* bn_scale,
                                 const float* bn_shift, float* bn_part, int bn_nparts);
int conv_nhwc_fwd_ring_nparts(int N, int H, int W, int R, int S, int sh, int sw, int ph, int pw, int variant);
void conv_nhwc_fwd_ring(int dtype, const void* x, const void* w, void* y, const void* zero, int N, int H, int W, int C,
                        int K, int R, int S, int sh, int sw, int ph, int pw, int variant, float* part, int nparts,
                        hipStream_t s);
bool conv3x3_halo_ok(int C, int K, int R, int S, int sh, int sw, int ph, int pw, int W);
int conv3x3_halo_nparts(int N, int H);
void conv3x3_halo(int dtype, const void* x, const void* w, void* y, const void* zero, int N, int H, int W, int C, int K,
                  float* part, int nparts, const void* bn_z, const float* bn_mean, const float* bn_scale,
                  const float* bn_shift, int bn_mode, float* bn_part, hipStream_t s);
int conv_nhwc_wgrad_ring_ok(int C, int K, int R, int S, int variant);
int64_t conv_nhwc_wgrad_ring_workspace(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                                       int variant, int dh, int dw);
void conv_nhwc_wgrad_ring(int dtype, const void* x, const void* dy, float* slab, int out_dtype, void* out, int accum,
                          int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                          const void* zero, int variant, hipStream_t s, int dh, int dw);
int64_t conv_nhwc_wgrad_workspace(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                                  int dh, int dw);
void conv_nhwc_wgrad(int dtype, const void* x, const void* dy, float* slab, int out_dtype, void* out, int accum, int N,
                     int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, const void* zero,
                     hipStream_t s, int dh, int dw);
int conv_stem_grid(int N, int H, int W, int R, int S, int ph, int pw);
void conv_stem_fwd(int dtype, const void* x, const void* w, void* y, int N, int H, int W, int C, int K, int R, int S,
                   int sh, int sw, int ph, int pw, float* part, int nparts, hipStream_t s);
int64_t conv_stem_wgrad_workspace(int N, int H, int W, int R, int S, int ph, int pw);
void conv_stem_wgrad(int dtype, const void* x, const void* dy, float* slab, int out_dtype, void* out, int accum, int N,
                     int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, hipStream_t s);
int layernorm_bwd_partials(int M);
void layernorm_forward(int dtype, const void* x, const void* gamma, const void* beta, int pt, void* y, float* mean,
                       float* rstd, int M, int D, float eps, hipStream_t s);
void layernorm_backward(int dtype, const void* x, const void* dy, const void* gamma, int pt, const float* mean,
                        const float* rstd, void* dx, float* part, void* dgamma, void* dbeta, int gdtype, int accum,
                        int M, int D, hipStream_t s);
void add_dropout_ln_forward(int dtype, const void* x, const void* h, const void* gamma, const void* beta, int pt,
                            void* y, void* s_out, uint8_t* mask, float* mean, float* rstd, int M, int D, float eps,
                            float p, uint64_t seed, const uint64_t* seed_base, hipStream_t s);
void add_dropout_ln_backward(int dtype, const void* s_in, const void* dy, const void* gamma, int pt, const float* mean,
                             const float* rstd, const uint8_t* mask, float p, void* ds, void* dh, float* part,
                             float* hpart, void* dgamma, void* dbeta, int gdtype, int accum, int M, int D,
                             hipStream_t s);
void column_sum_partials(int gdtype, const float* part, int nb, int ncol, void* out, int accum, hipStream_t s);
void gelu_forward(int dtype, const void* x, void* y, int64_t n, hipStream_t s);
void gelu_backward(int dtype, const void* x, const void* dy, void* dx, int64_t n, hipStream_t s);
void gelu_backward_colpart(int dtype, const void* x, const void* dy, void* dx, float* part, int M, int N,
                           hipStream_t s);
int gelu_colpart_blocks(int M, int N);
void softmax_forward(int dtype, int log, const void* x, void* y, int M, int L, float scale, hipStream_t s);
void softmax_backward(int dtype, int log, const void* y, const void* dy, void* dx, int M, int L, float scale,
                      hipStream_t s);
void dropout_forward(int dtype, const void* x, void* y, uint8_t* mask, int64_t n, float p, uint64_t seed,
                     const uint64_t* seed_base, hipStream_t s);
void dropout_backward(int dtype, const void* dy, const uint8_t* mask, void* dx, int64_t n, float p, hipStream_t s);
int attention_max_seq();
void attention_forward(int dtype, const void* qkv, const float* kmask, void* out, float* lse, int S, int B, int H,
                       int D, float scale, float p, uint64_t seed, const uint64_t* seed_base, hipStream_t s);
void attention_backward(int dtype, const void* qkv, const float* kmask, const void* out, const void* dout,
                        const float* lse, float* delta, void* dqkv, int S, int B, int H, int D, float scale, float p,
                        uint64_t seed, const uint64_t* seed_base, hipStream_t s);
void flat_adam(int dtype, int mode, void* w, const void* g, float* mean, float* var, float* w32, int64_t n, float lr,
               float beta1, float beta2, float eps, float wd, float eta, float rescale, float clip, const float* hp,
               hipStream_t s);
void lamb_update(int dtype, void* w, const void* g, float* mean, float* var, float* w32, float* upd,
                 const void* chunks, int nchunks, float* nrm, int nseg, float lr, float beta1, float beta2, float eps,
                 float bc1, float bc2, float wd, float rescale, float clip, float lb, float ub, const float* hp,
                 hipStream_t s);
void seg_sumsq(int dtype, const void* x, const void* chunks, int nchunks, float* out, int nseg, hipStream_t s);
void all_finite(int dtype, const void* x, int64_t n, float scale, int* flag, int init, hipStream_t s);
void pool_nhwc_forward(int dtype, int is_max, const void* x, void* y, uint8_t* arg, int N, int H, int W, int C,
                       int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int cip, hipStream_t s,
                       const float* scale, const float* shift);
int bn_pool_bwd_blocks();
void bn_pool_backward(int dtype, const void* x, const void* dy, const uint8_t* arg, void* dx, const float* gamma,
                      const float* mean, const float* invstd, const float* fscale, const float* fshift, float* part,
                      float* dgamma, float* dbeta, float* coef, int N, int H, int W, int C, int Ho, int Wo, int kh,
                      int kw, int sh, int sw, int ph, int pw, int fix_gamma, int training, int accum,
                      hipStream_t s);
void pool_nhwc_backward(int dtype, int is_max, const void* dy, const uint8_t* arg, void* dx, int N, int H, int W,
                        int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int cip,
                        hipStream_t s);
void deform_im2col(int dtype, const void* x, const void* off, const void* msk, void* cols, int N, int C, int H, int W,
                   int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int dg,
                   int rows, hipStream_t s);
void deform_col2im(int dtype, const void* off, const void* msk, const void* gcols, float* gx, int N, int C, int H,
                   int W, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int dh, int dw, int dg,
                   int rows, hipStream_t s);
void deform_col2im_coord(int dtype, const void* x, const void* off, const void* msk, const void* gcols, void* goff,
                         void* gmsk, int N, int C, int H, int W, int Ho, int Wo, int kh, int kw, int sh, int sw,
                         int ph, int pw, int dh, int dw, int dg, int rows, hipStream_t s);
void deform_im2col_nhwc(int dtype, const void* x, const void* off, const void* msk, void* cols, const int* g,
                        int ld_off, int ld_msk, hipStream_t s);
void deform_bwd_nhwc(int dtype, const void* x, const void* off, const void* msk, const void* gcols, float* gx,
                     void* goff, void* gmsk, const int* g, int ld_off, int ld_msk, hipStream_t s);
void conv_dw_fwd(int dtype, const void* x, const void* wt, const float* bias, void* y, const int* gm, hipStream_t s);
void conv_dw_dgrad(int dtype, const void* dy, const void* wt, void* dx, const int* gm, hipStream_t s);
void conv_dw_wgrad(int dtype, const void* x, const void* dy, float* slab, int nslice, int out_dtype, void* out,
                   int accum, const int* gm, hipStream_t s);
int ssd_loss_blocks(int rows);
void ssd_loss_fwd(int dtype, const void* cls, const void* loc, const float* cls_t, const float* loc_t,
                  const float* loc_m, int rows, int C1, float lambd, float* part, float* out, hipStream_t s);
void ssd_loss_bwd(int dtype, const void* cls, const void* loc, const float* cls_t, const float* loc_t,
                  const float* loc_m, const float* stats, const float* gout, int rows, int C1, float lambd, void* dcls,
                  void* dloc, hipStream_t s);
void multibox_target(int dtype, const float* anchors, const float* labels, const void* cls_pred, float* loc_target,
                     float* loc_mask, float* cls_target, float* match_iou, int* match_gt, uint32_t* key, int B, int A,
                     int L, int W, int C, float thr, float ignore_label, float neg_ratio, float neg_thresh,
                     int min_neg, float v0, float v1, float v2, float v3, hipStream_t s);
void slab_reduce(int out_dtype, float* slab, int splits, int64_t n, void* out, int accum, hipStream_t s);
void twobit_quantize(int dtype, const void* g, float* res, void* packed, int64_t n, float thr, hipStream_t s);
void twobit_dequantize_sum(const void* packed, int64_t row_bytes, int nrows, int64_t n, float thr, float* out,
                           hipStream_t s);
int conv_pw_stream_ok(int kin, int nout);
int conv_pw_stream_grid(int M, int kin, int nout, int ncu, int add);
int conv_pw_stream_slices(int kin, int nout);
void weight_taps_t(int elem_bytes, const void* w, void* out, int K, int RS, int C, int n, const int* src,
                   const int64_t* base, const int64_t* rstride, hipStream_t s);
void conv_pw_stream(int dtype, const void* x, const void* w, void* y, const void* zero, int M, int kin, int nout,
                    float* part, int grid, hipStream_t s, const void* addend, int wt, const void* bn_z,
                    const uint8_t* bn_mask, const float* bn_mean, const float* bn_scale, const float* bn_shift,
                    int bn_mode, const uint8_t* addend_mask);
int conv_pw_stream_bnb_ok(int kin, int nout, int add, int mode);
void conv_gen(int dtype, int mode, const void* src, const void* wsrc, const float* bias, void* dst, const int* geom,
              int splits, hipStream_t s);
void rnn_fwd_seq(int dtype, int mode, const float* gx, const void* h0, const float* c0, const void* whh,
                 const float* bhh, void* out, int ldo, float* cseq, float* save, int Tn, int N, int H, int reverse,
                 hipStream_t s);
void rnn_bwd_seq(int dtype, int mode, const void* whhT, const void* dy, int ldy, const float* dhT,
                 const float* save, const float* cseq, const float* c0, const void* h0, const void* out, int ldo,
                 void* dgh, void* dgx, float* dc, float* dhd, float* dh0, int Tn, int N, int H, int reverse,
                 hipStream_t s);
}  // namespace mxamd

using namespace mxamd;

template <typename T>
static inline T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
static inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
static inline hipStream_t S_(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static void check_launch(const char* name) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(name) + ": " + hipGetErrorString(e));
}

PYBIND11_MODULE(_hip_kernels, m) {
  m.doc() = "gfx950 HIP kernels for mxnet_maintenance_amd";
  m.attr("arch") = "gfx950";

  m.def("bn_partials_rows", &bn_partials_rows);
  m.def("bn_tail_ds_rows", &bn_tail_ds_rows);
  m.def("bn_nhwc_stats", [](int dt, uintptr_t x, uintptr_t center, uintptr_t part, int64_t R, int C, uintptr_t s) {
    int nblk = bn_nhwc_stats(dt, P<const void>(x), P<const float>(center), P<float>(part), R, C, S(s), 512);
    check_launch("bn_nhwc_stats");
    return nblk;
  });
  m.def("embedding_forward", [](int dt, int it, uintptr_t idx, uintptr_t w, uintptr_t y, int64_t n, int V, int C,
                                uintptr_t s) {
    embedding_forward(dt, it, P<const void>(idx), P<const void>(w), P<void>(y), n, V, C, S(s));
    check_launch("embedding_forward");
  });
  m.def("embedding_backward", [](int dt, int it, uintptr_t idx, uintptr_t dy, uintptr_t acc, uintptr_t touched,
                                 int odt, uintptr_t grad, int accum, int64_t n, int V, int C, uintptr_t s) {
    embedding_backward(dt, it, P<const void>(idx), P<const void>(dy), P<float>(acc), P<uint8_t>(touched), odt,
                       P<void>(grad), accum, n, V, C, S(s));
    check_launch("embedding_backward");
  });
  m.def("csr_dot_dense", [](int dt, uintptr_t indptr, uintptr_t indices, uintptr_t vals, uintptr_t rhs, uintptr_t out,
                            int64_t M, int64_t K, int N, uintptr_t s) {
    csr_dot_dense(dt, P<const int64_t>(indptr), P<const int64_t>(indices), P<const void>(vals), P<const void>(rhs),
                  P<void>(out), M, K, N, S(s));
    check_launch("csr_dot_dense");
  });
  m.def("csrT_dot_dense", [](int dt, uintptr_t indptr, uintptr_t indices, uintptr_t vals, uintptr_t rhs,
                             uintptr_t slot, uintptr_t out32, int64_t M, int64_t K, int N, uintptr_t s) {
    csrT_dot_dense(dt, P<const int64_t>(indptr), P<const int64_t>(indices), P<const void>(vals), P<const void>(rhs),
                   P<const int64_t>(slot), P<float>(out32), M, K, N, S(s));
    check_launch("csrT_dot_dense");
  });
  m.def("int8_gemm", [](uintptr_t a, uintptr_t b, uintptr_t c, int M, int N, int K, uintptr_t s) {
    int8_gemm(P<const int8_t>(a), P<const int8_t>(b), P<int32_t>(c), M, N, K, S(s));
    check_launch("int8_gemm");
  });
  m.def("colsum_partials", [](int64_t R, int C) { return colsum_partials(R, C); });
  m.def("colsum_rows", [](int dt, uintptr_t x, uintptr_t zeros, uintptr_t part, int64_t R, int C, int odt,
                          uintptr_t out, int accum, uintptr_t s) {
    colsum_rows(dt, P<const void>(x), P<const float>(zeros), P<float>(part), R, C, odt, P<void>(out), accum, S(s));
    check_launch("colsum_rows");
  });
  m.def("twobit_quantize", [](int dt, uintptr_t g, uintptr_t res, uintptr_t packed, int64_t n, float thr,
                              uintptr_t s) {
    twobit_quantize(dt, P<void>(g), P<float>(res), P<void>(packed), n, thr, S(s));
    check_launch("twobit_quantize");
  });
  m.def("twobit_dequantize_sum", [](uintptr_t packed, int64_t row_bytes, int nrows, int64_t n, float thr,
                                    uintptr_t out, uintptr_t s) {
    twobit_dequantize_sum(P<void>(packed), row_bytes, nrows, n, thr, P<float>(out), S(s));
    check_launch("twobit_dequantize_sum");
  });
  // bias_lowp: the bias is in the operand dtype (read as such in the epilogue), else fp32
  m.def("gemm_nt", [](int dt, uintptr_t a, uintptr_t b, uintptr_t bias, uintptr_t addend, uintptr_t c, int out_f32,
                      int M, int N, int K, int lda, int ldb, int ldc, int act, int cfg, int splits, uintptr_t ws,
                      uintptr_t s, int bias_lowp) {
    gemm_nt(dt, P<void>(a), P<void>(b), P<void>(bias), P<void>(addend), P<void>(c), out_f32, M, N, K, lda, ldb, ldc,
            act, cfg, splits, P<float>(ws), S(s), bias_lowp);
    check_launch("gemm_nt");
  }, py::arg("dt"), py::arg("a"), py::arg("b"), py::arg("bias"), py::arg("addend"), py::arg("c"), py::arg("out_f32"),
     py::arg("M"), py::arg("N"), py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("act"),
     py::arg("cfg"), py::arg("splits"), py::arg("ws"), py::arg("s"), py::arg("bias_lowp") = 0);
  // streaming 1x1 convolution for small reductions (src/kernels/conv_pw.hip)
  m.def("weight_taps_t", [](int eb, uintptr_t w, uintptr_t out, int K, int RS, int C, std::vector<int> src,
                            std::vector<int64_t> base, std::vector<int64_t> rstride, uintptr_t s) {
    if (src.size() != base.size() || src.size() != rstride.size()) throw std::runtime_error("weight_taps_t: table sizes");
    weight_taps_t(eb, P<const void>(w), P<void>(out), K, RS, C, static_cast<int>(src.size()), src.data(), base.data(),
                  rstride.data(), S(s));
    check_launch("weight_taps_t");
  });
  m.def("conv_pw_stream_ok", &conv_pw_stream_ok);
  m.def("conv_pw_stream_slices", &conv_pw_stream_slices);
  m.def("conv_pw_stream_grid", [](int M, int kin, int nout, int ncu, int add) {
    return conv_pw_stream_grid(M, kin, nout, ncu, add);
  }, pybind11::arg("M"), pybind11::arg("kin"), pybind11::arg("nout"), pybind11::arg("ncu"), pybind11::arg("add") = 0);
  m.def("conv_pw_stream", [](int dt, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t zero, int M, int kin, int nout,
                             uintptr_t part, int grid, uintptr_t s, uintptr_t addend, int wt, uintptr_t bn_z,
                             uintptr_t bn_mask, uintptr_t bn_mean, uintptr_t bn_scale, uintptr_t bn_shift, int bn_mode,
                             uintptr_t addend_mask) {
    conv_pw_stream(dt, P<const void>(x), P<const void>(w), P<void>(y), P<const void>(zero), M, kin, nout,
                   P<float>(part), grid, S(s), P<const void>(addend), wt, P<const void>(bn_z), P<const uint8_t>(bn_mask),
                   P<const float>(bn_mean), P<const float>(bn_scale), P<const float>(bn_shift), bn_mode,
                   P<const uint8_t>(addend_mask));
    check_launch("conv_pw_stream");
  }, pybind11::arg("dt"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("zero"),
     pybind11::arg("M"), pybind11::arg("kin"), pybind11::arg("nout"), pybind11::arg("part"), pybind11::arg("grid"),
     pybind11::arg("s"), pybind11::arg("addend"), pybind11::arg("wt") = 0, pybind11::arg("bn_z") = 0,
     pybind11::arg("bn_mask") = 0, pybind11::arg("bn_mean") = 0, pybind11::arg("bn_scale") = 0,
     pybind11::arg("bn_shift") = 0, pybind11::arg("bn_mode") = 0, pybind11::arg("addend_mask") = 0);
  m.def("conv_pw_stream_bnb_ok", &conv_pw_stream_bnb_ok);
  // general implicit-GEMM convolution: grouped / dilated / 1-3-D / fp32 / transposed (src/kernels/conv_gen.hip)
  m.def("conv_gen", [](int dt, int mode, uintptr_t src, uintptr_t wsrc, uintptr_t bias, uintptr_t dst,
                       std::vector<int> geom, int splits, uintptr_t s) {
    if (geom.size() != 22) throw std::runtime_error("conv_gen: geometry needs 22 ints");
    conv_gen(dt, mode, P<const void>(src), P<const void>(wsrc), P<const float>(bias), P<void>(dst), geom.data(),
             splits, S(s));
    check_launch("conv_gen");
  });
  // fused recurrent layers: one (layer, direction) over a whole sequence (src/kernels/rnn.hip)
  m.def("rnn_fwd_seq", [](int dt, int mode, uintptr_t gx, uintptr_t h0, uintptr_t c0, uintptr_t whh, uintptr_t bhh,
                          uintptr_t out, int ldo, uintptr_t cseq, uintptr_t save, int T, int N, int H, int reverse,
                          uintptr_t s) {
    rnn_fwd_seq(dt, mode, P<const float>(gx), P<const void>(h0), P<const float>(c0), P<const void>(whh),
                P<const float>(bhh), P<void>(out), ldo, P<float>(cseq), P<float>(save), T, N, H, reverse, S(s));
    check_launch("rnn_fwd_seq");
  });
  m.def("rnn_bwd_seq", [](int dt, int mode, uintptr_t whhT, uintptr_t dy, int ldy, uintptr_t dhT, uintptr_t save,
                          uintptr_t cseq, uintptr_t c0, uintptr_t h0, uintptr_t out, int ldo, uintptr_t dgh,
                          uintptr_t dgx, uintptr_t dc, uintptr_t dhd, uintptr_t dh0, int T, int N, int H, int reverse,
                          uintptr_t s) {
    rnn_bwd_seq(dt, mode, P<const void>(whhT), P<const void>(dy), ldy, P<const float>(dhT), P<const float>(save),
                P<const float>(cseq), P<const float>(c0), P<const void>(h0), P<const void>(out), ldo, P<void>(dgh),
                P<void>(dgx), P<float>(dc), P<float>(dhd), P<float>(dh0), T, N, H, reverse, S(s));
    check_launch("rnn_bwd_seq");
  });
  m.def("gemm_nt_tile_n", &gemm_nt_tile_n);
  m.def("gemm_nt_tile_m", &gemm_nt_tile_m);
  m.def("slab_reduce", [](int odt, uintptr_t slab, int splits, int64_t n, uintptr_t out, int accum, uintptr_t s) {
    slab_reduce(odt, P<float>(slab), splits, n, P<void>(out), accum, S(s));
    check_launch("slab_reduce");
  });
  // deformable convolution (NCHW): geometry g = [N, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg(, rows)]
  // rows = 1: columns [N*Ho*Wo][C*kh*kw] (the MFMA GEMM operand layout), else [N][C*kh*kw][Ho*Wo]
  m.def("deform_im2col", [](int dt, uintptr_t x, uintptr_t off, uintptr_t msk, uintptr_t cols, std::vector<int> g,
                            uintptr_t s) {
    if (g.size() != 15 && g.size() != 16) throw std::runtime_error("deform_im2col: geometry needs 15 or 16 ints");
    const int rows = g.size() == 16 ? g[15] : 0;
    deform_im2col(dt, P<void>(x), P<void>(off), P<void>(msk), P<void>(cols), g[0], g[1], g[2], g[3], g[4], g[5], g[6],
                  g[7], g[8], g[9], g[10], g[11], g[12], g[13], g[14], rows, S(s));
    check_launch("deform_im2col");
  });
  m.def("deform_col2im", [](int dt, uintptr_t off, uintptr_t msk, uintptr_t gcols, uintptr_t gx, std::vector<int> g,
                            uintptr_t s) {
    if (g.size() != 15 && g.size() != 16) throw std::runtime_error("deform_col2im: geometry needs 15 or 16 ints");
    const int rows = g.size() == 16 ? g[15] : 0;
    deform_col2im(dt, P<void>(off), P<void>(msk), P<void>(gcols), P<float>(gx), g[0], g[1], g[2], g[3], g[4], g[5],
                  g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13], g[14], rows, S(s));
    check_launch("deform_col2im");
  });
  m.def("deform_col2im_coord", [](int dt, uintptr_t x, uintptr_t off, uintptr_t msk, uintptr_t gcols, uintptr_t goff,
                                  uintptr_t gmsk, std::vector<int> g, uintptr_t s) {
    if (g.size() != 15 && g.size() != 16) throw std::runtime_error("deform_col2im_coord: geometry needs 15 or 16 ints");
    const int rows = g.size() == 16 ? g[15] : 0;
    deform_col2im_coord(dt, P<void>(x), P<void>(off), P<void>(msk), P<void>(gcols), P<void>(goff), P<void>(gmsk),
                        g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13], g[14],
                        rows, S(s));
    check_launch("deform_col2im_coord");
  });
  // channels-last deformable conv (same 15-int geometry; x / offsets / mask / gradients NHWC, offsets and
  // mask rows ld_off / ld_msk elements apart)
  m.def("deform_im2col_nhwc", [](int dt, uintptr_t x, uintptr_t off, uintptr_t msk, uintptr_t cols, std::vector<int> g,
                                 int ld_off, int ld_msk, uintptr_t s) {
    if (g.size() != 15) throw std::runtime_error("deform_im2col_nhwc: geometry needs 15 ints");
    deform_im2col_nhwc(dt, P<void>(x), P<void>(off), P<void>(msk), P<void>(cols), g.data(), ld_off, ld_msk, S(s));
    check_launch("deform_im2col_nhwc");
  });
  m.def("deform_bwd_nhwc", [](int dt, uintptr_t x, uintptr_t off, uintptr_t msk, uintptr_t gcols, uintptr_t gx,
                              uintptr_t goff, uintptr_t gmsk, std::vector<int> g, int ld_off, int ld_msk, uintptr_t s) {
    if (g.size() != 15) throw std::runtime_error("deform_bwd_nhwc: geometry needs 15 ints");
    deform_bwd_nhwc(dt, P<void>(x), P<void>(off), P<void>(msk), P<void>(gcols), P<float>(gx), P<void>(goff),
                    P<void>(gmsk), g.data(), ld_off, ld_msk, S(s));
    check_launch("deform_bwd_nhwc");
  });
  // depthwise NHWC conv; geometry g = [N, H, W, C, Ho, Wo, R, S, sh, sw, ph, pw, dh, dw]; wt = [R*S][C]
  m.def("conv_dw_fwd", [](int dt, uintptr_t x, uintptr_t wt, uintptr_t bias, uintptr_t y, std::vector<int> g,
                          uintptr_t s) {
    if (g.size() != 14) throw std::runtime_error("conv_dw_fwd: geometry needs 14 ints");
    conv_dw_fwd(dt, P<void>(x), P<void>(wt), P<float>(bias), P<void>(y), g.data(), S(s));
    check_launch("conv_dw_fwd");
  });
  m.def("conv_dw_dgrad", [](int dt, uintptr_t dy, uintptr_t wt, uintptr_t dx, std::vector<int> g, uintptr_t s) {
    if (g.size() != 14) throw std::runtime_error("conv_dw_dgrad: geometry needs 14 ints");
    conv_dw_dgrad(dt, P<void>(dy), P<void>(wt), P<void>(dx), g.data(), S(s));
    check_launch("conv_dw_dgrad");
  });
  m.def("conv_dw_wgrad", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t slab, int nslice, int out_dt, uintptr_t out,
                            int accum, std::vector<int> g, uintptr_t s) {
    if (g.size() != 14) throw std::runtime_error("conv_dw_wgrad: geometry needs 14 ints");
    conv_dw_wgrad(dt, P<void>(x), P<void>(dy), P<float>(slab), nslice, out_dt, P<void>(out), accum, g.data(), S(s));
    check_launch("conv_dw_wgrad");
  });
  // fused SSD training loss (detection.hip): softmax-CE (ignore -1, valid normalisation) + smooth-L1
  m.def("ssd_loss_blocks", &ssd_loss_blocks);
  m.def("ssd_loss_fwd", [](int dt, uintptr_t cls, uintptr_t loc, uintptr_t ct, uintptr_t lt, uintptr_t lm, int rows,
                           int C1, float lambd, uintptr_t part, uintptr_t out, uintptr_t s) {
    ssd_loss_fwd(dt, P<void>(cls), P<void>(loc), P<float>(ct), P<float>(lt), P<float>(lm), rows, C1, lambd,
                 P<float>(part), P<float>(out), S(s));
    check_launch("ssd_loss_fwd");
  });
  m.def("ssd_loss_bwd", [](int dt, uintptr_t cls, uintptr_t loc, uintptr_t ct, uintptr_t lt, uintptr_t lm,
                           uintptr_t stats, uintptr_t gout, int rows, int C1, float lambd, uintptr_t dcls, uintptr_t dloc,
                           uintptr_t s) {
    ssd_loss_bwd(dt, P<void>(cls), P<void>(loc), P<float>(ct), P<float>(lt), P<float>(lm), P<float>(stats),
                 P<float>(gout), rows, C1, lambd, P<void>(dcls), P<void>(dloc), S(s));
    check_launch("ssd_loss_bwd");
  });
  m.def("multibox_target", [](int dt, uintptr_t anchors, uintptr_t labels, uintptr_t cls_pred, uintptr_t loc_target,
                              uintptr_t loc_mask, uintptr_t cls_target, uintptr_t match_iou, uintptr_t match_gt,
                              uintptr_t key, int B, int A, int L, int W, int C, float thr, float ignore_label,
                              float neg_ratio, float neg_thresh, int min_neg, float v0, float v1, float v2, float v3,
                              uintptr_t s) {
    multibox_target(dt, P<float>(anchors), P<float>(labels), P<void>(cls_pred), P<float>(loc_target),
                    P<float>(loc_mask), P<float>(cls_target), P<float>(match_iou), P<int>(match_gt),
                    P<uint32_t>(key), B, A, L, W, C, thr, ignore_label, neg_ratio, neg_thresh, min_neg, v0, v1, v2,
                    v3, S(s));
    check_launch("multibox_target");
  });
  // mask: optional uint8 ReLU bitmask (one byte per 8 elements) written by the add+relu tail
  m.def("bn_nhwc_forward", [](int dt, uintptr_t x, uintptr_t add, uintptr_t y, uintptr_t mask, uintptr_t g, uintptr_t b,
                              uintptr_t center, uintptr_t part, uintptr_t mean, uintptr_t inv, uintptr_t var,
                              uintptr_t scale, uintptr_t shift, int64_t R, int C, float eps, int training, int relu,
                              int fix_gamma, float momentum, uintptr_t mm_upd, uintptr_t mv_upd, int ext_nblk,
                              uintptr_t s) {
    bn_nhwc_forward(dt, P<void>(x), P<void>(add), P<void>(y), P<uint8_t>(mask), P<float>(g), P<float>(b), P<float>(center),
                    P<float>(part), P<float>(mean), P<float>(inv), P<float>(var), P<float>(scale), P<float>(shift), R,
                    C, eps, training, relu, fix_gamma, momentum, P<float>(mm_upd), P<float>(mv_upd), ext_nblk, S(s));
    check_launch("bn_nhwc_forward");
  });
  // relu_mode: 0 none, 1 mask from y, 2 mask recomputed from x*fscale+fshift, 3 from the forward's bitmask;
  // accum: += into dgamma/dbeta
  m.def("bn_nhwc_backward", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t y, uintptr_t mask, uintptr_t dx,
                               uintptr_t dz,
                               uintptr_t g, uintptr_t mean, uintptr_t inv, uintptr_t fscale, uintptr_t fshift,
                               uintptr_t part, uintptr_t dgamma, uintptr_t dbeta, uintptr_t coef, int64_t R, int C,
                               int relu_mode, int fix_gamma, int training, int accum, uintptr_t s, int ext_nblk,
                               uintptr_t ds_z, uintptr_t ds_mean, uintptr_t ds_part) {
    bn_nhwc_backward(dt, P<void>(x), P<void>(dy), P<void>(y), P<uint8_t>(mask), P<void>(dx), P<void>(dz), P<float>(g), P<float>(mean),
                     P<float>(inv), P<float>(fscale), P<float>(fshift), P<float>(part), P<float>(dgamma),
                     P<float>(dbeta), P<float>(coef), R, C, relu_mode, fix_gamma, training, accum, S(s), ext_nblk,
                     P<const void>(ds_z), P<const float>(ds_mean), P<float>(ds_part));
    check_launch("bn_nhwc_backward");
  }, py::arg("dt"), py::arg("x"), py::arg("dy"), py::arg("y"), py::arg("mask"), py::arg("dx"), py::arg("dz"),
     py::arg("g"), py::arg("mean"), py::arg("inv"), py::arg("fscale"), py::arg("fshift"), py::arg("part"),
     py::arg("dgamma"), py::arg("dbeta"), py::arg("coef"), py::arg("R"), py::arg("C"), py::arg("relu_mode"),
     py::arg("fix_gamma"), py::arg("training"), py::arg("accum"), py::arg("stream"), py::arg("ext_nblk") = 0,
     py::arg("ds_z") = 0, py::arg("ds_mean") = 0, py::arg("ds_part") = 0);
  m.def("softmax_ce_forward", [](int dt, int li, uintptr_t logits, uintptr_t label, uintptr_t loss, uintptr_t lse,
                                 int N, int K, uintptr_t s) {
    softmax_ce_forward(dt, li, P<void>(logits), P<void>(label), P<float>(loss), P<float>(lse), N, K, S(s));
    check_launch("softmax_ce_forward");
  });
  m.def("softmax_ce_backward", [](int dt, int li, uintptr_t logits, uintptr_t label, uintptr_t lse, uintptr_t gout,
                                  uintptr_t dlogits, int N, int K, uintptr_t s) {
    softmax_ce_backward(dt, li, P<void>(logits), P<void>(label), P<float>(lse), P<float>(gout), P<void>(dlogits), N,
                        K, S(s));
    check_launch("softmax_ce_backward");
  });
  m.def("relu_forward", [](int dt, uintptr_t x, uintptr_t y, int64_t n, uintptr_t s) {
    relu_forward(dt, P<void>(x), P<void>(y), n, S(s));
    check_launch("relu_forward");
  });
  m.def("relu_backward", [](int dt, uintptr_t y, uintptr_t dy, uintptr_t dx, int64_t n, uintptr_t s) {
    relu_backward(dt, P<void>(y), P<void>(dy), P<void>(dx), n, S(s));
    check_launch("relu_backward");
  });
  m.def("pointwise_binary", [](int dt, int op, uintptr_t a, uintptr_t b, uintptr_t out, int64_t n, int mode,
                               int64_t row, std::vector<int64_t> shape, std::vector<int64_t> sa,
                               std::vector<int64_t> sb, uintptr_t s) {
    if (shape.size() != sa.size() || shape.size() != sb.size()) throw std::runtime_error("pointwise_binary: rank");
    pointwise_binary(dt, op, P<void>(a), P<void>(b), P<void>(out), n, mode, row, static_cast<int>(shape.size()),
                     shape.data(), sa.data(), sb.data(), S(s));
    check_launch("pointwise_binary");
  });
  m.def("gap_nhwc_forward", [](int dt, uintptr_t x, uintptr_t y, int N, int HW, int C, uintptr_t s) {
    gap_nhwc_forward(dt, P<void>(x), P<void>(y), N, HW, C, S(s));
    check_launch("gap_nhwc_forward");
  });
  m.def("gap_nhwc_backward", [](int dt, uintptr_t dy, uintptr_t dx, int N, int HW, int C, uintptr_t s) {
    gap_nhwc_backward(dt, P<void>(dy), P<void>(dx), N, HW, C, S(s));
    check_launch("gap_nhwc_backward");
  });
  m.def("flat_sgd", [](int dt, uintptr_t w, uintptr_t g, uintptr_t mom, uintptr_t w32, int64_t n, float lr,
                       float wd, float momentum, float rescale, float clip, uintptr_t s) {
    flat_sgd(dt, P<void>(w), P<void>(g), P<float>(mom), P<float>(w32), n, lr, wd, momentum, rescale, clip, nullptr,
             S(s));
    check_launch("flat_sgd");
  });
  // overload with a trailing device hyper-parameter pointer (hp[0] = lr), for HIP-graph-captured steps
  m.def("flat_sgd", [](int dt, uintptr_t w, uintptr_t g, uintptr_t mom, uintptr_t w32, int64_t n, float lr,
                       float wd, float momentum, float rescale, float clip, uintptr_t s, uintptr_t hp) {
    flat_sgd(dt, P<void>(w), P<void>(g), P<float>(mom), P<float>(w32), n, lr, wd, momentum, rescale, clip,
             P<float>(hp), S(s));
    check_launch("flat_sgd");
  });
  // variant: 0 heuristic tile, 1..4 = (BCO, BK) in (128,64) (128,32) (64,64) (64,32)
  m.def("conv_nhwc_fwd", [](int dt, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int N, int H, int W,
                            int C, int K, int R, int Sf, int sh, int sw, int ph, int pw, int variant, uintptr_t s) {
    conv_nhwc_fwd(dt, P<void>(x), P<void>(w), P<float>(bias), P<void>(y), N, H, W, C, K, R, Sf, sh, sw, ph, pw,
                  variant, S(s));
    check_launch("conv_nhwc_fwd");
  });
  m.def("conv_nhwc_fwd_glds", [](int dt, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, uintptr_t zero, int N,
                                 int H, int W, int C, int K, int R, int Sf, int sh, int sw, int ph, int pw, int bco,
                                 uintptr_t s, uintptr_t bn_z, uintptr_t bn_mean, uintptr_t bn_scale,
                                 uintptr_t bn_shift, uintptr_t bn_part, int bn_nparts) {
    conv_nhwc_fwd_glds(dt, P<void>(x), P<void>(w), P<float>(bias), P<void>(y), P<void>(zero), N, H, W, C, K, R, Sf,
                       sh, sw, ph, pw, bco, S(s), P<void>(bn_z), P<float>(bn_mean), P<float>(bn_scale),
                       P<float>(bn_shift), P<float>(bn_part), bn_nparts);
    check_launch("conv_nhwc_fwd_glds");
  }, py::arg("dtype"), py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("zero"), py::arg("N"),
     py::arg("H"), py::arg("W"), py::arg("C"), py::arg("K"), py::arg("R"), py::arg("S"), py::arg("sh"),
     py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("bco"), py::arg("stream"), py::arg("bn_z") = 0,
     py::arg("bn_mean") = 0, py::arg("bn_scale") = 0, py::arg("bn_shift") = 0, py::arg("bn_part") = 0,
     py::arg("bn_nparts") = 0);
  // BN-backward partials per channel of a glds launch over M output pixels (per phase for the phase kernel)
  m.def("conv_glds_bwd_nparts", &conv_glds_bwd_nparts);
  // the sub-pixel phases of a strided data gradient, one launch, written in place into dX
  m.def("conv_nhwc_dgrad_phases_glds",
        [](int dt, uintptr_t dy, uintptr_t w, uintptr_t dx, uintptr_t zero, int N, int Hi, int Wi, int Cin, int Cout,
           int Ho, int Wo, int stride, std::vector<int> ph, std::vector<int> pw, std::vector<int> R,
           std::vector<int> Sf, std::vector<int> pad_h, std::vector<int> pad_w, std::vector<int64_t> w_off,
           std::vector<int> zph, std::vector<int> zpw, int bco, uintptr_t s, uintptr_t bn_z, uintptr_t bn_mean,
           uintptr_t bn_scale, uintptr_t bn_shift, uintptr_t bn_part, int bn_nparts) {
          const size_t n = ph.size();
          if (pw.size() != n || R.size() != n || Sf.size() != n || pad_h.size() != n || pad_w.size() != n ||
              w_off.size() != n || zph.size() != zpw.size())
            throw std::runtime_error("conv_nhwc_dgrad_phases_glds: per-phase lists differ in length");
          conv_nhwc_dgrad_phases_glds(dt, P<void>(dy), P<void>(w), P<void>(dx), P<void>(zero), N, Hi, Wi, Cin, Cout,
                                      Ho, Wo, stride, (int)n, ph.data(), pw.data(), R.data(), Sf.data(),
                                      pad_h.data(), pad_w.data(), w_off.data(), (int)zph.size(), zph.data(),
                                      zpw.data(), bco, S(s), P<void>(bn_z), P<float>(bn_mean), P<float>(bn_scale),
                                      P<float>(bn_shift), P<float>(bn_part), bn_nparts);
          check_launch("conv_nhwc_dgrad_phases_glds");
        },
        py::arg("dtype"), py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("zero"), py::arg("N"), py::arg("Hi"),
        py::arg("Wi"), py::arg("Cin"), py::arg("Cout"), py::arg("Ho"), py::arg("Wo"), py::arg("stride"),
        py::arg("ph"), py::arg("pw"), py::arg("R"), py::arg("S"), py::arg("pad_h"), py::arg("pad_w"),
        py::arg("w_off"), py::arg("zph"), py::arg("zpw"), py::arg("bco"), py::arg("stream"), py::arg("bn_z") = 0,
        py::arg("bn_mean") = 0, py::arg("bn_scale") = 0, py::arg("bn_shift") = 0, py::arg("bn_part") = 0,
        py::arg("bn_nparts") = 0);
  // 512-thread big-tile kernel: variant 0..3 = 256x256, 128x256, 64x512, 256x128 (co x pix), 4 / 5 =
  // 128x256 / 256x128 at two workgroups per CU;
  // part (optional): channel-major [2][K][nparts] BatchNorm sum / sum-of-squares partials of y
  // few-channel stride-2 stems (conv_stem.hip): Cin <= 4, Cout = 64, kernel up to 8x8
  m.def("conv_stem_grid", &conv_stem_grid);
  m.def("conv_stem_wgrad_workspace", &conv_stem_wgrad_workspace);
  m.def("conv_stem_fwd", [](int dt, uintptr_t x, uintptr_t w, uintptr_t y, int N, int H, int W, int C, int K, int R,
                            int Sf, int sh, int sw, int ph, int pw, uintptr_t part, int nparts, uintptr_t s) {
    conv_stem_fwd(dt, P<void>(x), P<void>(w), P<void>(y), N, H, W, C, K, R, Sf, sh, sw, ph, pw, P<float>(part),
                  nparts, S(s));
    check_launch("conv_stem_fwd");
  });
  m.def("conv_stem_wgrad", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t slab, int odt, uintptr_t out, int accum,
                              int N, int H, int W, int C, int K, int R, int Sf, int sh, int sw, int ph, int pw,
                              uintptr_t s) {
    conv_stem_wgrad(dt, P<void>(x), P<void>(dy), P<float>(slab), odt, P<void>(out), accum, N, H, W, C, K, R, Sf, sh,
                    sw, ph, pw, S(s));
    check_launch("conv_stem_wgrad");
  });
  m.def("conv_nhwc_fwd_big_nparts", &conv_nhwc_fwd_big_nparts);
  m.def("conv_nhwc_fwd_big_bwd_nparts", &conv_nhwc_fwd_big_bwd_nparts);
  // bn (optional): (z, mean, scale, shift, mask, mode, part, nparts) -- BN-backward statistics of y
  m.def("conv_nhwc_fwd_big", [](int dt, uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, uintptr_t zero, int N,
                                int H, int W, int C, int K, int R, int Sf, int sh, int sw, int ph, int pw, int variant,
                                uintptr_t part, int nparts, uintptr_t addend, uintptr_t s, uintptr_t bz,
                                uintptr_t bmean, uintptr_t bscale, uintptr_t bshift, uintptr_t bmask, int bmode,
                                uintptr_t bpart, int bnparts, int up, int dh, int dw) {
    conv_nhwc_fwd_big(dt, P<void>(x), P<void>(w), P<float>(bias), P<void>(y), P<void>(zero), N, H, W, C, K, R, Sf, sh,
                      sw, ph, pw, variant, P<float>(part), nparts, P<void>(addend), S(s), P<void>(bz), P<float>(bmean),
                      P<float>(bscale), P<float>(bshift), P<uint8_t>(bmask), bmode, P<float>(bpart), bnparts, up, dh,
                      dw);
    check_launch("conv_nhwc_fwd_big");
  }, py::arg("dt"), py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("zero"), py::arg("N"),
     py::arg("H"), py::arg("W"), py::arg("C"), py::arg("K"), py::arg("R"), py::arg("S"), py::arg("sh"),
     py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("variant"), py::arg("part"), py::arg("nparts"),
     py::arg("addend"), py::arg("stream"), py::arg("bn_z") = 0, py::arg("bn_mean") = 0, py::arg("bn_scale") = 0,
     py::arg("bn_shift") = 0, py::arg("bn_mask") = 0, py::arg("bn_mode") = 0, py::arg("bn_part") = 0,
     py::arg("bn_nparts") = 0, py::arg("up") = 0, py::arg("dh") = 1, py::arg("dw") = 1);
  // persistent LDS-DMA ring kernel (conv_ring.hip): variant 0..5 = 128x128x4, 256x128x3, 128x256x3, 64x256x4,
  // 256x256x2, 64x128x4 (co x pix x stages); part as above
  m.def("conv_nhwc_fwd_ring_nparts", &conv_nhwc_fwd_ring_nparts);
  m.def("conv_nhwc_fwd_ring", [](int dt, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t zero, int N, int H, int W,
                                 int C, int K, int R, int Sf, int sh, int sw, int ph, int pw, int variant, uintptr_t part,
                                 int nparts, uintptr_t s) {
    conv_nhwc_fwd_ring(dt, P<void>(x), P<void>(w), P<void>(y), P<void>(zero), N, H, W, C, K, R, Sf, sh, sw, ph, pw,
                       variant, P<float>(part), nparts, S(s));
    check_launch("conv_nhwc_fwd_ring");
  });
  // 3x3 stride-1 C = K = 64 halo-tile conv (conv_halo.hip): resident weights, one patch per 4 rows
  m.def("conv3x3_halo_ok", &conv3x3_halo_ok);
  m.def("conv3x3_halo_nparts", &conv3x3_halo_nparts);
  m.def("conv3x3_halo", [](int dt, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t zero, int N, int H, int W, int C,
                           int K, uintptr_t part, int nparts, uintptr_t bn_z, uintptr_t bn_mean, uintptr_t bn_scale,
                           uintptr_t bn_shift, int bn_mode, uintptr_t bn_part, uintptr_t s) {
    conv3x3_halo(dt, P<void>(x), P<void>(w), P<void>(y), P<void>(zero), N, H, W, C, K, P<float>(part), nparts,
                 P<void>(bn_z), P<float>(bn_mean), P<float>(bn_scale), P<float>(bn_shift), bn_mode, P<float>(bn_part),
                 S(s));
    check_launch("conv3x3_halo");
  }, py::arg("dt"), py::arg("x"), py::arg("w"), py::arg("y"), py::arg("zero"), py::arg("N"), py::arg("H"),
     py::arg("W"), py::arg("C"), py::arg("K"), py::arg("part"), py::arg("nparts"), py::arg("bn_z") = 0,
     py::arg("bn_mean") = 0, py::arg("bn_scale") = 0, py::arg("bn_shift") = 0, py::arg("bn_mode") = 0,
     py::arg("bn_part") = 0, py::arg("s") = 0);
  m.def("conv_nhwc_wgrad_workspace", &conv_nhwc_wgrad_workspace, py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"),
        py::arg("K"), py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("dh") = 1, py::arg("dw") = 1);
  // weight gradient on the LDS-DMA ring (variants 1..5, see conv_wgrad.hip)
  m.def("conv_nhwc_wgrad_ring_ok", &conv_nhwc_wgrad_ring_ok);
  m.def("conv_nhwc_wgrad_ring_workspace", &conv_nhwc_wgrad_ring_workspace, py::arg("N"), py::arg("H"), py::arg("W"),
        py::arg("C"), py::arg("K"), py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"),
        py::arg("pw"), py::arg("variant"), py::arg("dh") = 1, py::arg("dw") = 1);
  m.def("conv_nhwc_wgrad_ring", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t slab, int odt, uintptr_t out,
                                   int accum, int N, int H, int W, int C, int K, int R, int Sf, int sh, int sw, int ph,
                                   int pw, uintptr_t zero, int variant, uintptr_t s, int dh, int dw) {
    conv_nhwc_wgrad_ring(dt, P<void>(x), P<void>(dy), P<float>(slab), odt, P<void>(out), accum, N, H, W, C, K, R, Sf,
                         sh, sw, ph, pw, P<void>(zero), variant, S(s), dh, dw);
    check_launch("conv_nhwc_wgrad_ring");
  }, py::arg("dt"), py::arg("x"), py::arg("dy"), py::arg("slab"), py::arg("odt"), py::arg("out"), py::arg("accum"),
     py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("K"), py::arg("R"), py::arg("S"), py::arg("sh"),
     py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("zero"), py::arg("variant"), py::arg("stream"),
     py::arg("dh") = 1, py::arg("dw") = 1);
  // zero: 0 -> register-staged kernel, else a >=128-byte zero page -> LDS-DMA kernel
  m.def("conv_nhwc_wgrad", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t slab, int odt, uintptr_t out, int accum,
                              int N, int H, int W, int C, int K, int R, int Sf, int sh, int sw, int ph, int pw,
                              uintptr_t zero, uintptr_t s, int dh, int dw) {
    conv_nhwc_wgrad(dt, P<void>(x), P<void>(dy), P<float>(slab), odt, P<void>(out), accum, N, H, W, C, K, R, Sf, sh,
                    sw, ph, pw, P<void>(zero), S(s), dh, dw);
    check_launch("conv_nhwc_wgrad");
  }, py::arg("dt"), py::arg("x"), py::arg("dy"), py::arg("slab"), py::arg("odt"), py::arg("out"), py::arg("accum"),
     py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("K"), py::arg("R"), py::arg("S"), py::arg("sh"),
     py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("zero"), py::arg("stream"), py::arg("dh") = 1,
     py::arg("dw") = 1);
  m.def("layernorm_bwd_partials", &layernorm_bwd_partials);
  // pt: gamma / beta in the activation dtype (else fp32)
  m.def("layernorm_forward", [](int dt, uintptr_t x, uintptr_t g, uintptr_t b, uintptr_t y, uintptr_t mean,
                                uintptr_t rstd, int M, int D, float eps, uintptr_t s, int pt) {
    layernorm_forward(dt, P<void>(x), P<void>(g), P<void>(b), pt, P<void>(y), P<float>(mean), P<float>(rstd), M, D,
                      eps, S(s));
    check_launch("layernorm_forward");
  }, py::arg("dtype"), py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("y"), py::arg("mean"),
     py::arg("rstd"), py::arg("M"), py::arg("D"), py::arg("eps"), py::arg("stream"), py::arg("pt") = 0);
  m.def("layernorm_backward", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t g, uintptr_t mean, uintptr_t rstd,
                                 uintptr_t dx, uintptr_t part, uintptr_t dg, uintptr_t db, int gdt, int accum, int M,
                                 int D, uintptr_t s, int pt) {
    layernorm_backward(dt, P<void>(x), P<void>(dy), P<void>(g), pt, P<float>(mean), P<float>(rstd), P<void>(dx),
                       P<float>(part), P<void>(dg), P<void>(db), gdt, accum, M, D, S(s));
    check_launch("layernorm_backward");
  }, py::arg("dtype"), py::arg("x"), py::arg("dy"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
     py::arg("dx"), py::arg("part"), py::arg("dgamma"), py::arg("dbeta"), py::arg("gdtype"), py::arg("accum"),
     py::arg("M"), py::arg("D"), py::arg("stream"), py::arg("pt") = 0);
  // y = LayerNorm(x + dropout(h)) and its backward (ds, dh = dropout'(ds), dgamma / dbeta)
  m.def("add_dropout_ln_forward", [](int dt, uintptr_t x, uintptr_t h, uintptr_t g, uintptr_t b, int pt, uintptr_t y,
                                     uintptr_t sum, uintptr_t mask, uintptr_t mean, uintptr_t rstd, int M, int D,
                                     float eps, float p, uint64_t seed, uintptr_t seed_base, uintptr_t s) {
    add_dropout_ln_forward(dt, P<void>(x), P<void>(h), P<void>(g), P<void>(b), pt, P<void>(y), P<void>(sum),
                           P<uint8_t>(mask), P<float>(mean), P<float>(rstd), M, D, eps, p, seed,
                           P<uint64_t>(seed_base), S(s));
    check_launch("add_dropout_ln_forward");
  });
  m.def("add_dropout_ln_backward", [](int dt, uintptr_t sum, uintptr_t dy, uintptr_t g, int pt, uintptr_t mean,
                                      uintptr_t rstd, uintptr_t mask, float p, uintptr_t ds, uintptr_t dh,
                                      uintptr_t part, uintptr_t hpart, uintptr_t dg, uintptr_t db, int gdt, int accum,
                                      int M, int D, uintptr_t s) {
    add_dropout_ln_backward(dt, P<void>(sum), P<void>(dy), P<void>(g), pt, P<float>(mean), P<float>(rstd),
                            P<uint8_t>(mask), p, P<void>(ds), P<void>(dh), P<float>(part), P<float>(hpart),
                            P<void>(dg), P<void>(db), gdt, accum, M, D, S(s));
    check_launch("add_dropout_ln_backward");
  });
  m.def("column_sum_partials", [](int gdt, uintptr_t part, int nb, int ncol, uintptr_t out, int accum, uintptr_t s) {
    column_sum_partials(gdt, P<float>(part), nb, ncol, P<void>(out), accum, S(s));
    check_launch("column_sum_partials");
  });
  m.def("gelu_forward", [](int dt, uintptr_t x, uintptr_t y, int64_t n, uintptr_t s) {
    gelu_forward(dt, P<void>(x), P<void>(y), n, S(s));
    check_launch("gelu_forward");
  });
  m.def("gelu_colpart_blocks", &gelu_colpart_blocks);
  m.def("gelu_backward_colpart", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t dx, uintptr_t part, int M, int N,
                                    uintptr_t s) {
    gelu_backward_colpart(dt, P<void>(x), P<void>(dy), P<void>(dx), P<float>(part), M, N, S(s));
    check_launch("gelu_backward_colpart");
  });
  m.def("gelu_backward", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t dx, int64_t n, uintptr_t s) {
    gelu_backward(dt, P<void>(x), P<void>(dy), P<void>(dx), n, S(s));
    check_launch("gelu_backward");
  });
  m.def("softmax_forward", [](int dt, int log, uintptr_t x, uintptr_t y, int M, int L, float scale, uintptr_t s) {
    softmax_forward(dt, log, P<void>(x), P<void>(y), M, L, scale, S(s));
    check_launch("softmax_forward");
  });
  m.def("softmax_backward", [](int dt, int log, uintptr_t y, uintptr_t dy, uintptr_t dx, int M, int L, float scale,
                               uintptr_t s) {
    softmax_backward(dt, log, P<void>(y), P<void>(dy), P<void>(dx), M, L, scale, S(s));
    check_launch("softmax_backward");
  });
  m.def("dropout_forward", [](int dt, uintptr_t x, uintptr_t y, uintptr_t mask, int64_t n, float p, uint64_t seed,
                              uintptr_t s) {
    dropout_forward(dt, P<void>(x), P<void>(y), P<uint8_t>(mask), n, p, seed, nullptr, S(s));
    check_launch("dropout_forward");
  });
  // overload: seed_base = device uint64 counter mixed into the seed (fresh masks on every graph replay)
  m.def("dropout_forward", [](int dt, uintptr_t x, uintptr_t y, uintptr_t mask, int64_t n, float p, uint64_t seed,
                              uintptr_t s, uintptr_t seed_base) {
    dropout_forward(dt, P<void>(x), P<void>(y), P<uint8_t>(mask), n, p, seed, P<uint64_t>(seed_base), S(s));
    check_launch("dropout_forward");
  });
  m.def("attention_max_seq", []() { return attention_max_seq(); });
  m.def("attention_forward", [](int dt, uintptr_t qkv, uintptr_t kmask, uintptr_t out, uintptr_t lse, int S, int B,
                                int H, int D, float scale, float p, uint64_t seed, uintptr_t seed_base, uintptr_t s) {
    attention_forward(dt, P<const void>(qkv), P<const float>(kmask), P<void>(out), P<float>(lse), S, B, H, D, scale, p,
                      seed, P<const uint64_t>(seed_base), S_(s));
    check_launch("attention_forward");
  });
  m.def("attention_backward", [](int dt, uintptr_t qkv, uintptr_t kmask, uintptr_t out, uintptr_t dout, uintptr_t lse,
                                 uintptr_t delta, uintptr_t dqkv, int S, int B, int H, int D, float scale, float p,
                                 uint64_t seed, uintptr_t seed_base, uintptr_t s) {
    attention_backward(dt, P<const void>(qkv), P<const float>(kmask), P<const void>(out), P<const void>(dout),
                       P<const float>(lse), P<float>(delta), P<void>(dqkv), S, B, H, D, scale, p, seed,
                       P<const uint64_t>(seed_base), S_(s));
    check_launch("attention_backward");
  });
  m.def("dropout_backward", [](int dt, uintptr_t dy, uintptr_t mask, uintptr_t dx, int64_t n, float p, uintptr_t s) {
    dropout_backward(dt, P<void>(dy), P<uint8_t>(mask), P<void>(dx), n, p, S(s));
    check_launch("dropout_backward");
  });
  // mode 0: Adam (wd folded into the gradient), 1: AdamW (decoupled, eta-scaled)
  m.def("flat_adam", [](int dt, int mode, uintptr_t w, uintptr_t g, uintptr_t mean, uintptr_t var, uintptr_t w32,
                        int64_t n, float lr, float b1, float b2, float eps, float wd, float eta, float rescale,
                        float clip, uintptr_t s) {
    flat_adam(dt, mode, P<void>(w), P<void>(g), P<float>(mean), P<float>(var), P<float>(w32), n, lr, b1, b2, eps, wd,
              eta, rescale, clip, nullptr, S(s));
    check_launch("flat_adam");
  });
  m.def("flat_adam", [](int dt, int mode, uintptr_t w, uintptr_t g, uintptr_t mean, uintptr_t var, uintptr_t w32,
                        int64_t n, float lr, float b1, float b2, float eps, float wd, float eta, float rescale,
                        float clip, uintptr_t s, uintptr_t hp) {
    flat_adam(dt, mode, P<void>(w), P<void>(g), P<float>(mean), P<float>(var), P<float>(w32), n, lr, b1, b2, eps, wd,
              eta, rescale, clip, P<float>(hp), S(s));
    check_launch("flat_adam");
  });
  m.def("lamb_update", [](int dt, uintptr_t w, uintptr_t g, uintptr_t mean, uintptr_t var, uintptr_t w32,
                          uintptr_t upd, uintptr_t chunks, int nchunks, uintptr_t nrm, int nseg, float lr, float b1,
                          float b2, float eps, float bc1, float bc2, float wd, float rescale, float clip, float lb,
                          float ub, uintptr_t s) {
    lamb_update(dt, P<void>(w), P<void>(g), P<float>(mean), P<float>(var), P<float>(w32), P<float>(upd),
                P<void>(chunks), nchunks, P<float>(nrm), nseg, lr, b1, b2, eps, bc1, bc2, wd, rescale, clip, lb, ub,
                nullptr, S(s));
    check_launch("lamb_update");
  });
  m.def("lamb_update", [](int dt, uintptr_t w, uintptr_t g, uintptr_t mean, uintptr_t var, uintptr_t w32,
                          uintptr_t upd, uintptr_t chunks, int nchunks, uintptr_t nrm, int nseg, float lr, float b1,
                          float b2, float eps, float bc1, float bc2, float wd, float rescale, float clip, float lb,
                          float ub, uintptr_t s, uintptr_t hp) {
    lamb_update(dt, P<void>(w), P<void>(g), P<float>(mean), P<float>(var), P<float>(w32), P<float>(upd),
                P<void>(chunks), nchunks, P<float>(nrm), nseg, lr, b1, b2, eps, bc1, bc2, wd, rescale, clip, lb, ub,
                P<float>(hp), S(s));
    check_launch("lamb_update");
  });
  m.def("seg_sumsq", [](int dt, uintptr_t x, uintptr_t chunks, int nchunks, uintptr_t out, int nseg, uintptr_t s) {
    seg_sumsq(dt, P<void>(x), P<void>(chunks), nchunks, P<float>(out), nseg, S(s));
    check_launch("seg_sumsq");
  });
  m.def("all_finite", [](int dt, uintptr_t x, int64_t n, float scale, uintptr_t flag, int init, uintptr_t s) {
    all_finite(dt, P<void>(x), n, scale, P<int>(flag), init, S(s));
    check_launch("all_finite");
  });
  m.def("pool_nhwc_forward", [](int dt, int is_max, uintptr_t x, uintptr_t y, uintptr_t arg, int N, int H, int W,
                                int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int cip,
                                uintptr_t s) {
    pool_nhwc_forward(dt, is_max, P<void>(x), P<void>(y), P<uint8_t>(arg), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw,
                      cip, S(s), nullptr, nullptr);
    check_launch("pool_nhwc_forward");
  });
  // backward of max_pool(relu(BatchNorm(x))): statistics gather, finalize, dx gather (pool_nhwc.hip)
  m.def("bn_pool_bwd_blocks", &bn_pool_bwd_blocks);
  m.def("bn_pool_backward", [](int dt, uintptr_t x, uintptr_t dy, uintptr_t arg, uintptr_t dx, uintptr_t gamma,
                               uintptr_t mean, uintptr_t invstd, uintptr_t fscale, uintptr_t fshift, uintptr_t part,
                               uintptr_t dgamma, uintptr_t dbeta, uintptr_t coef, int N, int H, int W, int C, int Ho,
                               int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int fix_gamma, int training,
                               int accum, uintptr_t s) {
    bn_pool_backward(dt, P<void>(x), P<void>(dy), P<uint8_t>(arg), P<void>(dx), P<float>(gamma), P<float>(mean),
                     P<float>(invstd), P<float>(fscale), P<float>(fshift), P<float>(part), P<float>(dgamma),
                     P<float>(dbeta), P<float>(coef), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, fix_gamma, training,
                     accum, S(s));
    check_launch("bn_pool_backward");
  });
  // 3x3 max pooling of relu(x * scale + shift): the stem's BatchNorm + ReLU folded into the pooling
  m.def("pool_nhwc_forward_bnrelu", [](int dt, uintptr_t x, uintptr_t y, uintptr_t arg, int N, int H, int W, int C,
                                       int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int cip,
                                       uintptr_t s, uintptr_t scale, uintptr_t shift) {
    pool_nhwc_forward(dt, 1, P<void>(x), P<void>(y), P<uint8_t>(arg), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, cip,
                      S(s), P<float>(scale), P<float>(shift));
    check_launch("pool_nhwc_forward_bnrelu");
  });
  m.def("pool_nhwc_backward", [](int dt, int is_max, uintptr_t dy, uintptr_t arg, uintptr_t dx, int N, int H, int W,
                                 int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph, int pw, int cip,
                                 uintptr_t s) {
    pool_nhwc_backward(dt, is_max, P<void>(dy), P<uint8_t>(arg), P<void>(dx), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph,
                       pw, cip, S(s));
    check_launch("pool_nhwc_backward");
  });
}
