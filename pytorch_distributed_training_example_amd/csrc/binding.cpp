// Python binding for the gfx950 kernels (pybind11 over at::Tensor).
//
// Thin by design: validates devices / dtypes / layouts, collects raw pointers, and calls the
// C-ABI launchers in kernels/*.hip on the current HIP stream (so the calls are ordered with
// PyTorch's own kernels and can be captured into a hipGraph). Every kernel lives in its own
// .hip translation unit; this file is the only one that includes the PyTorch headers.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cstring>
#include <map>
#include <vector>

extern "C" {
int pdt_sgd(int n, void* const* p, void* const* g, void* const* buf, void* const* copy, const int64_t* numel,
            int p_dtype, int g_dtype, float lr, const float* lr_ptr, float momentum, float dampening, float wd,
            int nesterov, int first, int maximize, const float* inv_scale, const float* found_inf, hipStream_t s);
int pdt_adam(int n, void* const* p, void* const* g, void* const* m, void* const* v, void* const* copy,
             const int64_t* numel, int p_dtype, int g_dtype, float lr, const float* lr_ptr, float beta1, float beta2,
             float eps, float wd, int decoupled, const float* step_ptr, float step_host, int maximize,
             const float* inv_scale, const float* found_inf, hipStream_t s);
int pdt_adadelta(int n, void* const* p, void* const* g, void* const* sa, void* const* ad, void* const* copy,
                 const int64_t* numel, int p_dtype, int g_dtype, float lr, const float* lr_ptr, float rho, float eps,
                 float wd, int maximize, const float* inv_scale, const float* found_inf, hipStream_t s);
int pdt_amp_unscale(int n, void* const* g, const int64_t* numel, int dtype, const float* inv_scale, float* found_inf,
                    hipStream_t s);
int pdt_amp_update(float* scale, int* growth_tracker, const float* found_inf, float growth, float backoff,
                   int interval, hipStream_t s);
int pdt_mt_scale(int n, void* const* x, const int64_t* numel, int dtype, const float* scale_ptr, float scale,
                 hipStream_t s);
int pdt_mt_copy(int n, void* const* src, void* const* dst, const int64_t* numel, int sdt, int ddt,
                const float* scale_ptr, float scale, hipStream_t s);
int pdt_l2norm_sq(int n, void* const* x, const int64_t* numel, int dtype, float* out, hipStream_t s);
int pdt_clip_coef(const float* sumsq, float max_norm, float* coef, float* norm, hipStream_t s);
int64_t pdt_bn_workspace_floats(int64_t M, int C);
int pdt_lenet_tail_fwd(const float* p1, const float* w2, const float* b2, const float* w3, const float* b3,
                       const float* fw1, const float* fb1, const float* fw2, const float* fb2, float slope, int N,
                       float* logits, uint8_t* code2, float* p2, float* h3, float* h4, hipStream_t s);
int64_t pdt_lenet_tail_ws_floats(int N);
int pdt_lenet_tail_bwd(const float* dl, const float* p1, const float* w2, const float* b2, const float* w3,
                       const float* b3, const float* fw1, const float* fb1, const float* fw2, const float* fb2,
                       float slope, int N, const uint8_t* code2, const float* p2, const float* h3, const float* h4,
                       float* ws, float* dp1, float* dw2, float* db2, float* dw3, float* db3, float* dfw1, float* dfb1,
                       float* dfw2, float* dfb2, hipStream_t s);
int pdt_bn_bwd_coef(const uint16_t* dy, const uint16_t* x, const uint8_t* mask, const float* gamma, const float* mean,
                    const float* invstd, int64_t M, int C, int relu, float* coef, float* dgamma, float* dbeta, float* ws,
                    unsigned* counters, hipStream_t s);
int pdt_bn_bwd_coef_tiles(const float* part, int T, const float* gamma, const float* invstd, int64_t M, int C,
                          float* coef, float* dgamma, float* dbeta, float* ws, hipStream_t s);
int pdt_conv1x1_bwd_fused_ok(int C4, int CW);
int pdt_conv1x1_bwd_fused_grid(int M, int C4, int CW);
int pdt_conv1x1_bwd_fused(const uint16_t* dy, const uint16_t* z, const uint8_t* mz, const float* mean, const float* A,
                          const float* B, const float* D, const uint16_t* wt, const uint16_t* xa, const uint16_t* bx,
                          const uint8_t* bm, const float* bmean, float* bpart, const float* xcoef, uint8_t* mask_out,
                          uint16_t* dxa, uint16_t* dw, float* ws, int M, int C4, int CW, hipStream_t s);
void pdt_conv1x1_bwd_fused_tune(int grid);
void pdt_bn_tune(int variant, int target_blocks, int u_fwd, int u_bwd);
int pdt_bn_fwd_train(const uint16_t* x, const uint16_t* res, const float* res_a, const float* res_b,
                     const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps, int64_t M, int C, int relu,
                     uint16_t* y, uint8_t* mask, float* mean, float* invstd, float* ws, unsigned* counters,
                     hipStream_t s);
int pdt_bn_fwd_eval(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta,
                    const float* running_mean, const float* running_var, float eps, int64_t M, int C, int relu,
                    uint16_t* y, float* ws, hipStream_t s);
int pdt_bn_bwd_train(const uint16_t* dy, const uint16_t* x, const uint8_t* mask, const float* gamma,
                     const float* mean, const float* invstd, int64_t M, int C, int relu, int has_res, uint16_t* dx,
                     uint16_t* dres, float* dgamma, float* dbeta, float* ws, unsigned* counters, hipStream_t s);
int pdt_ce_fwd(const void* logits, int dtype, const int64_t* target, int64_t N, int64_t V, float smoothing,
               int64_t ignore_index, float* loss, float* lse, hipStream_t s);
int pdt_ce_bwd(const void* logits, int dtype, const int64_t* target, const float* lse, const float* dloss,
               float dloss_scale, int64_t N, int64_t V, float smoothing, int64_t ignore_index, void* dlogits,
               hipStream_t s);
int64_t pdt_ln_workspace_floats(int64_t N, int D);
int pdt_ln_fwd(const void* x, const void* res, int dtype, const float* w, const float* b, void* y, void* sum_out,
               float* mean, float* rstd, int64_t N, int D, float eps, hipStream_t s);
int pdt_ln_fwd_fp8(const uint16_t* x, const uint16_t* res, const float* w, const float* b, uint16_t* sum_out,
                   uint8_t* yq, uint8_t* yqt, float* mean, float* rstd, int64_t N, int D, float eps,
                   const float* scale, float* amax, int striped, hipStream_t s);
int pdt_ln_bwd(const void* dy, const void* x, const void* dres, int dtype, const float* w, const float* mean,
               const float* rstd, void* dx, float* dw, float* db, int64_t N, int D, float* ws, hipStream_t s);
int pdt_attn_fwd(const uint16_t* q, const int64_t* qs, const uint16_t* k, const int64_t* ks, const uint16_t* v,
                 const int64_t* vs, uint16_t* o, const int64_t* os, float* lse, int B, int H, int T, int Dh,
                 int causal, float scale, hipStream_t s);
int pdt_attn_bwd(const uint16_t* dout, const int64_t* dos, const uint16_t* q, const int64_t* qs, const uint16_t* k,
                 const int64_t* ks, const uint16_t* v, const int64_t* vs, const uint16_t* o, const int64_t* os,
                 const float* lse, float* delta, uint16_t* dq, uint16_t* dk, uint16_t* dv, const int64_t* gs, int B,
                 int H, int T, int Dh, int causal, float scale, hipStream_t s);
int64_t pdt_gelu_workspace_floats(int64_t N, int D);
int pdt_bias_gelu_fwd(const void* x, int dtype, const void* bias, void* y, int64_t N, int D, int tanh_form,
                      hipStream_t s, int bias_bf16);
int pdt_bias_gelu_bwd(const void* dy, const void* x, int dtype, const void* bias, void* dx, void* dbias,
                      int64_t N, int D, int tanh_form, float* ws, hipStream_t s, int bias_bf16);
int pdt_bn_relu_maxpool_fwd_train(const uint16_t* x, const float* gamma, const float* beta, float* running_mean,
                                  float* running_var, float momentum, float eps, int N, int H, int W, int C,
                                  uint16_t* y, uint8_t* code, float* mean, float* invstd, float* ws,
                                  unsigned* counters, hipStream_t s);
int pdt_conv3x3s1_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int Ci, int Co,
                      hipStream_t s);
int pdt_conv3x3_flip_weights(const uint16_t* w, uint16_t* wf, int Co, int Ci, hipStream_t s);
int64_t pdt_conv3x3_wgrad_ws_floats(int N, int H, int W, int Ci, int Co, int* nsplit_out);
int pdt_conv3x3s1_wgrad(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, int N, int H, int W, int Ci,
                        int Co, hipStream_t s);
void pdt_conv3x3_wgrad_tune(int target_wgs, int co_tile);
int pdt_conv3x3s1_fwd_bnbwd(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* bn_x,
                            const uint8_t* bn_mask, const float* bn_mean, float* bn_part, int N, int H, int W, int Ci,
                            int Co, hipStream_t s);
int pdt_conv3x3s2_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, int N, int H, int W, int Ci,
                      int Co, hipStream_t s);
int pdt_conv3x3s2_dgrad(const uint16_t* dy, const uint16_t* wf, uint16_t* dx, const uint16_t* bn_x,
                        const uint8_t* bn_mask, const float* bn_mean, float* bn_part, int N, int H, int W, int Ci,
                        int Co, hipStream_t s);
int pdt_conv3x3s2_dgrad_tiles(int N, int H, int W);
int64_t pdt_conv3x3s2_wgrad_ws_floats(int N, int H, int W, int Ci, int Co, int* nsplit_out);
int pdt_conv3x3s2_wgrad(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, int N, int H, int W, int Ci,
                        int Co, hipStream_t s);
int pdt_conv3x3s1_fwd_stats(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, int N, int H, int W,
                            int Ci, int Co, hipStream_t s);
int64_t pdt_stem_conv_wprep_elems();
int64_t pdt_stem_stats_parts(int N, int H, int W);
int pdt_stem_conv_fwd_stats(const uint16_t* x, const uint16_t* w, uint16_t* wp, uint16_t* y, float* part, int N, int H,
                            int W, hipStream_t s);
int64_t pdt_bn_parts_ws_floats(int P, int C);
int pdt_bn_relu_maxpool_fwd_train_parts(const float* part, int P, const uint16_t* x, const float* gamma,
                                        const float* beta, float* running_mean, float* running_var, float momentum,
                                        float eps, int N, int H, int W, int C, uint16_t* y, uint8_t* code, float* mean,
                                        float* invstd, float* ws, hipStream_t s);
int pdt_stem_conv_fwd(const uint16_t* x, const uint16_t* w, uint16_t* wp, uint16_t* y, int N, int H, int W,
                      hipStream_t s);
int64_t pdt_stem_wgrad_ws_floats();
int pdt_stem_conv_wgrad(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, int N, int H, int W,
                        hipStream_t s);
int pdt_stem_conv_wgrad_bn_pool(const uint16_t* x, const uint16_t* dyp, const uint8_t* code, const uint16_t* xb,
                                const float* coef, const float* mean, uint16_t* dw, float* ws, int N, int H, int W,
                                hipStream_t s);
int pdt_stem_conv_wgrad_bn(const uint16_t* x, const uint16_t* dz, const uint16_t* xb, const float* coef,
                           const float* mean, uint16_t* dw, float* ws, int N, int H, int W, hipStream_t s);
int pdt_maxpool3s2_bwd(const uint16_t* dy, const uint8_t* code, uint16_t* dz, int N, int H, int W, int C,
                       hipStream_t s);
int pdt_conv1x1_tile_rows();
int64_t pdt_conv1x1_wgrad_ws_floats(int M, int Ci, int Co, int* nsplit_out);
int64_t pdt_conv1x1_wgrad_seg_ws_floats(int M, int Ci, int co1, int co2, int* rows_out);
int pdt_conv1x1_wgrad_seg(const uint16_t* x, const uint16_t* dy1, int co1, const uint16_t* dy2, int co2, float* out,
                          float* ws, int M, int Ci, hipStream_t s);
int pdt_conv1x1_gemm_seg(const uint16_t* a1, int k1, const uint16_t* a2, int k2, int rep2, const uint16_t* b,
                         uint16_t* y, int M, int N, const uint16_t* bn_x, const uint8_t* bn_mask, const float* bn_mean,
                         float* bn_part, hipStream_t s);
int pdt_bn_alg_fix_s2(float* part, int T, const float* wg, const uint16_t* W, int C4, int CW, hipStream_t s);
int pdt_bn_alg_ds_part(float* part, const float* s1, const float* mean, const float* wg, const uint16_t* W, int C4,
                       int CW, hipStream_t s);
int pdt_bn_alg_small_gemm(const uint16_t* W, const uint16_t* Wt, const float* coef, const float* wg, float* G,
                          float* BWG, int C4, int CW, hipStream_t s);
int pdt_bn_alg_assemble(const uint16_t* W, const float* coef, const float* mean, const float* G, const float* wg,
                        const float* BWG, uint16_t* bcat, uint16_t* dW, int C4, int CW, int rep, hipStream_t s);
int pdt_conv1x1_wgrad(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, int M, int Ci, int Co,
                      hipStream_t s);
void pdt_conv1x1_wgrad_tune(int target_wgs, int variant, int interleave);
int pdt_conv1x1_gemm(const uint16_t* a, const uint16_t* b, uint16_t* y, const uint16_t* c, const uint8_t* cm,
                     float* part, int M, int K, int N, const uint16_t* bn_x, const uint8_t* bn_mask,
                     const float* bn_mean, float* bn_part, int c_s, int c_H, int c_W, const float* acoef,
                     hipStream_t s, int nostore);
void pdt_conv1x1_probe(int probe);
int pdt_conv1x1_persist(int mode);
int pdt_conv3x3_opt(int v);
int pdt_conv3x3s1_stats_tile_rows(int N, int H, int W, int Ci, int Co);
int pdt_conv3x3s1_bnbwd_tile_rows(int N, int H, int W, int Ci, int Co);
void pdt_bn_tiles_fused(int on);
void pdt_maxpool_bwd_v2(int on);
void pdt_pool_fwd_contig(int on);
void pdt_bn_apply_wgs(int n);
void pdt_bn_row_wgs(int n);
int pdt_gap_bwd_parts(int64_t M, int C);
int pdt_gap_bwd(const uint16_t* g, int N, int HW, int C, uint16_t* dy, const uint16_t* xb, const uint8_t* mask,
                const float* mean, float* part, hipStream_t s);
int pdt_weight_prep_max_items();
int pdt_weight_prep(const uint16_t* const* src, uint16_t* const* dst, const int* R, const int* C, const int* taps,
                    int n, hipStream_t s);
int pdt_conv1x1_gemm_apply(const uint16_t* a, const uint16_t* b, uint16_t* y, const uint16_t* res, const float* ab,
                           const float* rab, uint8_t* mask, int M, int K, int N, const float* acoef, hipStream_t s);
int pdt_maxpool_bn_parts(int N, int H);
int pdt_maxpool3s2_bwd_bn(const uint16_t* dy, const uint8_t* code, uint16_t* dz, int N, int H, int W, int C,
                          const uint16_t* x, const float* gamma, const float* mean, const float* invstd, uint16_t* dx,
                          float* dgamma, float* dbeta, float* part, float* ws, hipStream_t s);
int pdt_maxpool3s2_bwd_bn_coef(const uint16_t* dy, const uint8_t* code, uint16_t* dz, int N, int H, int W, int C,
                               const uint16_t* x, const float* gamma, const float* mean, const float* invstd,
                               float* coef, float* dgamma, float* dbeta, float* part, float* ws, hipStream_t s);
int pdt_bn_bwd_train_tiles(const float* part, int T, int BMt, const uint16_t* dy, const uint16_t* x,
                           const uint8_t* mask, const float* gamma, const float* mean, const float* invstd, int64_t M,
                           int C, int relu, int has_res, uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta,
                           float* ws, hipStream_t s);
int64_t pdt_bn_tiles_ws_floats(int T, int C);
int pdt_bn_fwd_train_tiles(const float* part, int T, int BMt, const uint16_t* x, const uint16_t* res,
                           const float* res_a, const float* res_b,
                           const float* gamma, const float* beta, float* running_mean, float* running_var,
                           float momentum, float eps, int64_t M, int C, int relu, uint16_t* y, uint8_t* mask,
                           float* mean, float* invstd, float* ws, hipStream_t s, uint16_t* sub_y, int sub_H,
                           int sub_W, int sub_s);
int pdt_fp8_cast_transpose(const uint16_t* x, int64_t M, int64_t K, const float* scale, uint8_t* out,
                           uint8_t* out_t, float* amax, int striped, hipStream_t s);
int pdt_fp8_update_scales(float* state, int n, int L, float margin_scale, int striped, hipStream_t s);
// fp8 state rows of at least this many floats carry 16 amax stripes (csrc/fp8_pack.h kAmaxRowMin)
constexpr int64_t kFp8StripedRow = 261;
inline int fp8_striped(const at::Tensor& row) { return row.numel() >= kFp8StripedRow ? 1 : 0; }
int64_t pdt_fp8_gelu_cast_workspace_floats(int64_t M, int D);
int pdt_fp8_gelu_cast(const uint16_t* h, const uint16_t* dg, const float* bias, int64_t M, int D, int tanh_form,
                      const float* scale, uint8_t* out, uint8_t* out_t, float* amax, float* part, int striped,
                      hipStream_t s);
int pdt_fp8_cast_multi(int n, const uint16_t* const* x, const int* M, const int* K, float* const* st,
                       const int* striped, uint8_t* const* out, uint8_t* const* out_t, hipStream_t s);
int pdt_colsum_finalize(const float* part, int nblk, int D, void* out, int odtype, hipStream_t s);
int pdt_fp8_cast_colsum(const uint16_t* x, int64_t M, int D, const float* scale, uint8_t* out, uint8_t* out_t,
                        float* amax, float* part, int striped, hipStream_t s);
int pdt_embedding_fwd(const int64_t* idx, const uint16_t* wte, const uint16_t* wpe, uint16_t* out, int64_t n, int T,
                      int D, int V, int* err, hipStream_t s);
int64_t pdt_embedding_bwd_ws_ints(int64_t n, int V);
int pdt_gemm_nt(const uint16_t* A, const uint16_t* B, uint16_t* C, uint16_t* G, const void* bias, int bias_f32,
                int epi, int tanh_form, int M, int N, int K, hipStream_t s);
int pdt_gemm_nt_fp8_ksplit(int M, int N, int K);
int pdt_gemm_nt_fp8(const uint8_t* A, const uint8_t* B, uint16_t* C, const float* sa, const float* sb,
                    const void* bias, int bias_f32, int epi, int M, int N, int K, float* ws, int ksplit, hipStream_t s);
int pdt_embedding_bwd(const int64_t* idx, const uint16_t* dout, uint16_t* dwte, uint16_t* dwpe, int* ws, int64_t n,
                      int B, int T, int V, int D, int* err, hipStream_t s);
int64_t pdt_p2p_flags_bytes();
int64_t pdt_p2p_data_bytes(int64_t cap);
int pdt_p2p_allreduce(const void* in, void* out, int64_t n, int dtype, char* const* data_ptrs,
                      uint32_t* const* flag_ptrs, int rank, int world, int64_t cap, float post_scale,
                      uint32_t* st, int algo, int max_blocks, double timeout_s, hipStream_t s);
int pdt_colsum(const void* x, int dtype, int64_t N, int D, void* out, int odtype, float* ws, hipStream_t s);
int pdt_slice_sum_bf16(const uint16_t* x, uint16_t* out, int S, int64_t n, hipStream_t s);
int pdt_subsample_gather(const uint16_t* x, uint16_t* xs, int N, int H, int W, int C, int s, hipStream_t st);
int pdt_subsample_scatter_add(const uint16_t* t, uint16_t* full, int N, int H, int W, int C, int s, hipStream_t st);
int pdt_lenet_stem_fwd(const float* x, const float* w, const float* b, int64_t N, float slope, float* y,
                       uint8_t* code, hipStream_t s);
int64_t pdt_lenet_stem_slab_floats(int64_t N, int ipb);
int pdt_lenet_stem_bwd(const float* dy, const uint8_t* code, const float* x, int64_t N, int ipb, float slope,
                       float* slab, float* dw, float* db, hipStream_t s);
int pdt_leaky_pool_fwd(const float* x, int64_t planes, int H, int W, float slope, float* y, uint8_t* code,
                       hipStream_t s);
int pdt_leaky_pool_bwd(const float* dy, const uint8_t* code, int64_t planes, int H, int W, float slope, float* dx,
                       hipStream_t s);
int pdt_softmax_nll_small(const void* logits, int dtype, const int64_t* target, int64_t N, int V, int mode,
                          float smoothing, float* loss, void* dlogits, float dscale, double* acc, hipStream_t s);
int pdt_mean_small(const float* v, int64_t n, float scale, float* out, hipStream_t s);
}

namespace {

using at::Tensor;

hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

int dcode(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return 0;
  if (t.scalar_type() == at::kBFloat16) return 1;
  TORCH_CHECK(false, "pdt: unsupported dtype ", t.scalar_type(), " (fp32 / bf16 only)");
}

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "pdt: ", name, " must be a GPU tensor");
}

bool dense(const Tensor& t) { return t.is_contiguous() || t.is_non_overlapping_and_dense(); }

const float* opt_fptr(const c10::optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat, "pdt: scalar tensors must be fp32");
  return t->data_ptr<float>();
}

struct Lists {
  std::vector<void*> ptrs;
  static Lists from(const std::vector<Tensor>& ts, const char* name, int expect_dtype, size_t n) {
    Lists l;
    if (ts.empty()) {
      l.ptrs.assign(n, nullptr);
      return l;
    }
    TORCH_CHECK(ts.size() == n, "pdt: list ", name, " has ", ts.size(), " tensors, expected ", n);
    for (const auto& t : ts) {
      check_cuda(t, name);
      TORCH_CHECK(dense(t), "pdt: ", name, " tensors must be dense");
      if (expect_dtype >= 0) TORCH_CHECK(dcode(t) == expect_dtype, "pdt: ", name, " dtype mismatch");
      l.ptrs.push_back(t.data_ptr());
    }
    return l;
  }
};

std::vector<int64_t> numels(const std::vector<Tensor>& ts) {
  std::vector<int64_t> n;
  n.reserve(ts.size());
  for (const auto& t : ts) n.push_back(t.numel());
  return n;
}

void check_same_numel(const std::vector<Tensor>& a, const std::vector<Tensor>& b, const char* name) {
  if (b.empty()) return;
  for (size_t i = 0; i < a.size(); ++i)
    TORCH_CHECK(a[i].numel() == b[i].numel() && (a[i].strides() == b[i].strides() || a[i].is_contiguous() ==
                b[i].is_contiguous()), "pdt: ", name, "[", i, "] shape/layout mismatch");
}

int uniform_dtype(const std::vector<Tensor>& ts) {
  TORCH_CHECK(!ts.empty(), "pdt: empty tensor list");
  const int d = dcode(ts[0]);
  for (const auto& t : ts) TORCH_CHECK(dcode(t) == d, "pdt: mixed dtypes in one tensor list");
  return d;
}

// ----------------------------------------------------------------------------- optimizers
void sgd(std::vector<Tensor> params, std::vector<Tensor> grads, std::vector<Tensor> bufs,
         std::vector<Tensor> copies, double lr, c10::optional<Tensor> lr_t, double momentum, double dampening,
         double wd, bool nesterov, bool first, bool maximize, c10::optional<Tensor> inv_scale,
         c10::optional<Tensor> found_inf) {
  if (params.empty()) return;
  const size_t n = params.size();
  const int pd = uniform_dtype(params), gd = uniform_dtype(grads);
  check_same_numel(params, grads, "grads");
  check_same_numel(params, bufs, "momentum_buffer");
  check_same_numel(params, copies, "model_copy");
  auto P = Lists::from(params, "params", pd, n), G = Lists::from(grads, "grads", gd, n),
       B = Lists::from(bufs, "momentum_buffer", 0, n), C = Lists::from(copies, "model_copy", 1, n);
  auto ne = numels(params);
  int rc = pdt_sgd((int)n, P.ptrs.data(), G.ptrs.data(), B.ptrs.data(), C.ptrs.data(), ne.data(), pd, gd, (float)lr,
                   opt_fptr(lr_t), (float)momentum, (float)dampening, (float)wd, nesterov, first, maximize,
                   opt_fptr(inv_scale), opt_fptr(found_inf), stream());
  TORCH_CHECK(rc == 0, "pdt_sgd failed");
}

void adam(std::vector<Tensor> params, std::vector<Tensor> grads, std::vector<Tensor> exp_avg,
          std::vector<Tensor> exp_avg_sq, std::vector<Tensor> copies, double lr, c10::optional<Tensor> lr_t,
          double beta1, double beta2, double eps, double wd, bool decoupled, c10::optional<Tensor> step_t,
          double step, bool maximize, c10::optional<Tensor> inv_scale, c10::optional<Tensor> found_inf) {
  if (params.empty()) return;
  const size_t n = params.size();
  const int pd = uniform_dtype(params), gd = uniform_dtype(grads);
  check_same_numel(params, grads, "grads");
  check_same_numel(params, exp_avg, "exp_avg");
  check_same_numel(params, exp_avg_sq, "exp_avg_sq");
  check_same_numel(params, copies, "model_copy");
  TORCH_CHECK(!exp_avg.empty() && !exp_avg_sq.empty(), "pdt_adam: states required");
  auto P = Lists::from(params, "params", pd, n), G = Lists::from(grads, "grads", gd, n),
       M = Lists::from(exp_avg, "exp_avg", 0, n), V = Lists::from(exp_avg_sq, "exp_avg_sq", 0, n),
       C = Lists::from(copies, "model_copy", 1, n);
  auto ne = numels(params);
  int rc = pdt_adam((int)n, P.ptrs.data(), G.ptrs.data(), M.ptrs.data(), V.ptrs.data(), C.ptrs.data(), ne.data(), pd,
                    gd, (float)lr, opt_fptr(lr_t), (float)beta1, (float)beta2, (float)eps, (float)wd, decoupled,
                    opt_fptr(step_t), (float)step, maximize, opt_fptr(inv_scale), opt_fptr(found_inf), stream());
  TORCH_CHECK(rc == 0, "pdt_adam failed");
}

void adadelta(std::vector<Tensor> params, std::vector<Tensor> grads, std::vector<Tensor> square_avg,
              std::vector<Tensor> acc_delta, std::vector<Tensor> copies, double lr, c10::optional<Tensor> lr_t,
              double rho, double eps, double wd, bool maximize, c10::optional<Tensor> inv_scale,
              c10::optional<Tensor> found_inf) {
  if (params.empty()) return;
  const size_t n = params.size();
  const int pd = uniform_dtype(params), gd = uniform_dtype(grads);
  check_same_numel(params, grads, "grads");
  check_same_numel(params, square_avg, "square_avg");
  check_same_numel(params, acc_delta, "acc_delta");
  check_same_numel(params, copies, "model_copy");
  auto P = Lists::from(params, "params", pd, n), G = Lists::from(grads, "grads", gd, n),
       S = Lists::from(square_avg, "square_avg", 0, n), A = Lists::from(acc_delta, "acc_delta", 0, n),
       C = Lists::from(copies, "model_copy", 1, n);
  auto ne = numels(params);
  int rc = pdt_adadelta((int)n, P.ptrs.data(), G.ptrs.data(), S.ptrs.data(), A.ptrs.data(), C.ptrs.data(), ne.data(),
                        pd, gd, (float)lr, opt_fptr(lr_t), (float)rho, (float)eps, (float)wd, maximize,
                        opt_fptr(inv_scale), opt_fptr(found_inf), stream());
  TORCH_CHECK(rc == 0, "pdt_adadelta failed");
}

// ----------------------------------------------------------------------------- amp / buffers
void amp_unscale(std::vector<Tensor> grads, Tensor inv_scale, Tensor found_inf) {
  if (grads.empty()) return;
  const int d = uniform_dtype(grads);
  auto G = Lists::from(grads, "grads", d, grads.size());
  auto ne = numels(grads);
  TORCH_CHECK(pdt_amp_unscale((int)grads.size(), G.ptrs.data(), ne.data(), d, inv_scale.data_ptr<float>(),
                              found_inf.data_ptr<float>(), stream()) == 0, "pdt_amp_unscale failed");
}

void amp_update(Tensor scale, Tensor growth_tracker, Tensor found_inf, double growth, double backoff, int64_t interval) {
  TORCH_CHECK(growth_tracker.scalar_type() == at::kInt, "growth_tracker must be int32");
  pdt_amp_update(scale.data_ptr<float>(), growth_tracker.data_ptr<int>(), found_inf.data_ptr<float>(), (float)growth,
                 (float)backoff, (int)interval, stream());
}

void mt_scale(std::vector<Tensor> xs, c10::optional<Tensor> scale_t, double scale) {
  if (xs.empty()) return;
  const int d = uniform_dtype(xs);
  auto X = Lists::from(xs, "x", d, xs.size());
  auto ne = numels(xs);
  TORCH_CHECK(pdt_mt_scale((int)xs.size(), X.ptrs.data(), ne.data(), d, opt_fptr(scale_t), (float)scale, stream()) == 0,
              "pdt_mt_scale failed");
}

void mt_copy(std::vector<Tensor> src, std::vector<Tensor> dst, c10::optional<Tensor> scale_t, double scale) {
  if (src.empty()) return;
  TORCH_CHECK(src.size() == dst.size(), "mt_copy: list size mismatch");
  check_same_numel(src, dst, "dst");
  const int sd = uniform_dtype(src), dd = uniform_dtype(dst);
  auto S = Lists::from(src, "src", sd, src.size()), D = Lists::from(dst, "dst", dd, dst.size());
  auto ne = numels(src);
  TORCH_CHECK(pdt_mt_copy((int)src.size(), S.ptrs.data(), D.ptrs.data(), ne.data(), sd, dd, opt_fptr(scale_t),
                          (float)scale, stream()) == 0, "pdt_mt_copy failed");
}

void l2norm_sq(std::vector<Tensor> xs, Tensor out) {
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 1, "l2norm_sq: out must be fp32");
  if (xs.empty()) {
    out.zero_();
    return;
  }
  const int d = uniform_dtype(xs);
  auto X = Lists::from(xs, "x", d, xs.size());
  auto ne = numels(xs);
  pdt_l2norm_sq((int)xs.size(), X.ptrs.data(), ne.data(), d, out.data_ptr<float>(), stream());
}

void clip_coef(Tensor sumsq, double max_norm, Tensor coef, c10::optional<Tensor> norm) {
  pdt_clip_coef(sumsq.data_ptr<float>(), (float)max_norm, coef.data_ptr<float>(),
                norm.has_value() ? norm->data_ptr<float>() : nullptr, stream());
}

// ----------------------------------------------------------------------------- batchnorm (NHWC bf16)
void check_nhwc_bf16(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "pdt bn: ", name, " must be bf16");
  if (t.dim() == 4) {
    TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), "pdt bn: ", name, " must be channels_last");
  } else {
    TORCH_CHECK(t.dim() == 2 && t.is_contiguous(), "pdt bn: ", name, " must be [M, C] contiguous or NHWC");
  }
}

int64_t bn_ws_floats(int64_t M, int64_t C) { return pdt_bn_workspace_floats(M, (int)C); }

// Self-resetting arrival counters of the BN reduce kernels (one per 64-channel chunk), one
// buffer per device, zeroed once at creation (first call happens before any graph capture).
unsigned* bn_counters(const Tensor& like) {
  static std::map<int, Tensor> bufs;
  const int dev = like.get_device();
  auto it = bufs.find(dev);
  if (it == bufs.end()) {
    it = bufs.emplace(dev, at::zeros({4096}, like.options().dtype(at::kInt))).first;
  }
  return reinterpret_cast<unsigned*>(it->second.data_ptr<int>());
}

// res_ab [2, C] (optional): the residual is a deferred BatchNorm's input, added as ab[0]*res + ab[1].
// apply = false: statistics only -> {undefined, undefined, mean, invstd, ab [2, C]} (the y = a x + b
// coefficients, for a consumer that applies them itself).
std::pair<const float*, const float*> res_ab_ptrs(const c10::optional<Tensor>& res_ab, int64_t C) {
  if (!res_ab.has_value() || !res_ab->defined()) return {nullptr, nullptr};
  TORCH_CHECK(res_ab->scalar_type() == at::kFloat && res_ab->is_contiguous() && res_ab->numel() == 2 * C &&
              res_ab->is_cuda(), "pdt bn: res_ab must be fp32 [2, C]");
  return {res_ab->data_ptr<float>(), res_ab->data_ptr<float>() + C};
}

std::vector<Tensor> bn_fwd_train(Tensor x, c10::optional<Tensor> res, c10::optional<Tensor> weight,
                                 c10::optional<Tensor> bias, c10::optional<Tensor> running_mean,
                                 c10::optional<Tensor> running_var, double momentum, double eps, bool relu,
                                 c10::optional<Tensor> res_ab, bool apply) {
  check_nhwc_bf16(x, "x");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 64 == 0 && C <= 64 * 4096, "pdt bn: C must be a multiple of 64");
  const auto rab = res_ab_ptrs(res_ab, C);
  Tensor y;
  if (apply) y = at::empty_like(x);
  Tensor mask;
  if (relu && apply) mask = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  auto ws = at::empty({bn_ws_floats(M, C)}, fopt);
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_nhwc_bf16(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes() && res->strides() == x.strides(), "pdt bn: residual layout mismatch");
    rp = reinterpret_cast<const uint16_t*>(res->data_ptr());
  }
  float* rm = running_mean.has_value() && running_mean->defined() ? running_mean->data_ptr<float>() : nullptr;
  float* rv = running_var.has_value() && running_var->defined() ? running_var->data_ptr<float>() : nullptr;
  int rc = pdt_bn_fwd_train(reinterpret_cast<const uint16_t*>(x.data_ptr()), rp, rab.first, rab.second,
                            opt_fptr(weight), opt_fptr(bias), rm, rv,
                            (float)momentum, (float)eps, M, (int)C, relu,
                            apply ? reinterpret_cast<uint16_t*>(y.data_ptr()) : nullptr,
                            (relu && apply) ? mask.data_ptr<uint8_t>() : nullptr, mean.data_ptr<float>(),
                            invstd.data_ptr<float>(), ws.data_ptr<float>(), bn_counters(x), stream());
  TORCH_CHECK(rc == 0, "pdt_bn_fwd_train failed: ", rc);
  if (!apply) return {Tensor(), Tensor(), mean, invstd, ws.narrow(0, bn_ws_floats(M, C) - 4 * C, 2 * C).view({2, C})};
  return {y, mask, mean, invstd};
}

// ResNet stem tail (train): BN + ReLU + MaxPool2d(3, 2, 1) -> {y_pooled, code, mean, invstd}
std::vector<Tensor> bn_relu_maxpool_fwd(Tensor x, c10::optional<Tensor> weight, c10::optional<Tensor> bias,
                                        c10::optional<Tensor> running_mean, c10::optional<Tensor> running_var,
                                        double momentum, double eps) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4, "bn_relu_maxpool: 4-D NHWC input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 64 == 0, "pdt bn: C must be a multiple of 64");
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  auto y = at::empty({N, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto code = at::empty({N * Ho * Wo * C}, x.options().dtype(at::kByte));
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  auto ws = at::empty({bn_ws_floats(N * H * W, C)}, fopt);
  float* rm = running_mean.has_value() && running_mean->defined() ? running_mean->data_ptr<float>() : nullptr;
  float* rv = running_var.has_value() && running_var->defined() ? running_var->data_ptr<float>() : nullptr;
  int rc = pdt_bn_relu_maxpool_fwd_train(reinterpret_cast<const uint16_t*>(x.data_ptr()), opt_fptr(weight),
                                         opt_fptr(bias), rm, rv, (float)momentum, (float)eps, (int)N, (int)H, (int)W,
                                         (int)C, reinterpret_cast<uint16_t*>(y.data_ptr()), code.data_ptr<uint8_t>(),
                                         mean.data_ptr<float>(), invstd.data_ptr<float>(), ws.data_ptr<float>(),
                                         bn_counters(x), stream());
  TORCH_CHECK(rc == 0, "pdt_bn_relu_maxpool_fwd_train failed");
  return {y, code, mean, invstd};
}

// The same with the statistics from stem_conv_fwd_stats's partials (no reduce pass over x).
std::vector<Tensor> bn_relu_maxpool_fwd_parts(Tensor x, Tensor part, c10::optional<Tensor> weight,
                                              c10::optional<Tensor> bias, c10::optional<Tensor> running_mean,
                                              c10::optional<Tensor> running_var, double momentum, double eps) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4, "bn_relu_maxpool: 4-D NHWC input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C == 64, "bn_relu_maxpool_fwd_parts: C == 64 (the stem)");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 1 &&
                  part.numel() % (2 * C + 1) == 0, "bn_relu_maxpool_fwd_parts: part [P * (2 C + 1)] f32");
  const int64_t P = part.numel() / (2 * C + 1);
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  auto y = at::empty({N, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto code = at::empty({N * Ho * Wo * C}, x.options().dtype(at::kByte));
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  auto ws = at::empty({pdt_bn_parts_ws_floats((int)P, (int)C)}, fopt);
  float* rm = running_mean.has_value() && running_mean->defined() ? running_mean->data_ptr<float>() : nullptr;
  float* rv = running_var.has_value() && running_var->defined() ? running_var->data_ptr<float>() : nullptr;
  int rc = pdt_bn_relu_maxpool_fwd_train_parts(part.data_ptr<float>(), (int)P,
                                               reinterpret_cast<const uint16_t*>(x.data_ptr()), opt_fptr(weight),
                                               opt_fptr(bias), rm, rv, (float)momentum, (float)eps, (int)N, (int)H,
                                               (int)W, (int)C, reinterpret_cast<uint16_t*>(y.data_ptr()),
                                               code.data_ptr<uint8_t>(), mean.data_ptr<float>(),
                                               invstd.data_ptr<float>(), ws.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "pdt_bn_relu_maxpool_fwd_train_parts failed: ", rc);
  return {y, code, mean, invstd};
}

// Global-average-pool gradient: g [N, C] bf16 -> dy [N, C, H, W] channels_last = g / (H W). With bn_x / bn_mask /
// bn_mean (the pooled tensor is a BatchNorm(+ReLU) output): also that BatchNorm's backward partials [2, T, C]
// (the input of bn_bwd_train_tiles); {dy} alone when the reduction does not apply to C.
std::vector<Tensor> gap_bwd(Tensor g, int64_t H, int64_t W, c10::optional<Tensor> bn_x, c10::optional<Tensor> bn_mask,
                            c10::optional<Tensor> bn_mean, bool bn_sum_only) {
  check_cuda(g, "g");
  TORCH_CHECK(g.dim() == 2 && g.scalar_type() == at::kBFloat16 && g.is_contiguous() && g.size(1) % 8 == 0,
              "gap_bwd: g [N, C] contiguous bf16, C % 8 == 0");
  const int64_t N = g.size(0), C = g.size(1), M = N * H * W;
  auto dy = at::empty({N, C, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool red = ((bn_x.has_value() && bn_x->defined()) || bn_sum_only) && pdt_gap_bwd_parts(M, (int)C) > 0;
  Tensor part;
  const uint16_t* xp = nullptr;
  const uint8_t* mp = nullptr;
  const float* mu = nullptr;
  if (red) {
    if (!bn_sum_only) {
      check_nhwc_bf16(*bn_x, "bn_x");
      TORCH_CHECK(bn_x->sizes() == dy.sizes(), "gap_bwd: bn_x must be [N, C, H, W]");
      xp = reinterpret_cast<const uint16_t*>(bn_x->data_ptr());
    }
    TORCH_CHECK(bn_mean.has_value() && bn_mean->defined() && bn_mean->scalar_type() == at::kFloat &&
                    bn_mean->numel() == C && bn_mean->is_cuda(), "gap_bwd: bn_mean fp32 [C]");
    if (bn_mask.has_value() && bn_mask->defined()) {
      TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() == M * C / 8, "gap_bwd: bn_mask uint8 [M C / 8]");
      mp = bn_mask->data_ptr<uint8_t>();
    }
    mu = bn_mean->data_ptr<float>();
    part = at::empty({2, pdt_gap_bwd_parts(M, (int)C), C}, g.options().dtype(at::kFloat));
  }
  const int rc = pdt_gap_bwd(reinterpret_cast<const uint16_t*>(g.data_ptr()), (int)N, (int)(H * W), (int)C,
                             reinterpret_cast<uint16_t*>(dy.data_ptr()), xp, mp, mu,
                             red ? part.data_ptr<float>() : nullptr, stream());
  TORCH_CHECK(rc == 0, "pdt_gap_bwd failed: ", rc);
  if (red) return {dy, part};
  return {dy};
}

Tensor maxpool3s2_bwd(Tensor dy, Tensor code, int64_t H, int64_t W) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc_bf16(dy, "dy");
  const int64_t N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1 && code.numel() == dy.numel(),
              "maxpool3s2_bwd: shape mismatch");
  auto dz = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  int rc = pdt_maxpool3s2_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), code.data_ptr<uint8_t>(),
                              reinterpret_cast<uint16_t*>(dz.data_ptr()), (int)N, (int)H, (int)W, (int)C, stream());
  TORCH_CHECK(rc == 0, "pdt_maxpool3s2_bwd failed");
  return dz;
}

Tensor bn_fwd_eval(Tensor x, c10::optional<Tensor> res, c10::optional<Tensor> weight, c10::optional<Tensor> bias,
                   Tensor running_mean, Tensor running_var, double eps, bool relu) {
  check_nhwc_bf16(x, "x");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  auto y = at::empty_like(x);
  auto ws = at::empty({2 * C}, x.options().dtype(at::kFloat));
  const uint16_t* rp = (res.has_value() && res->defined()) ? reinterpret_cast<const uint16_t*>(res->data_ptr()) : nullptr;
  int rc = pdt_bn_fwd_eval(reinterpret_cast<const uint16_t*>(x.data_ptr()), rp, opt_fptr(weight), opt_fptr(bias),
                           running_mean.data_ptr<float>(), running_var.data_ptr<float>(), (float)eps, M, (int)C, relu,
                           reinterpret_cast<uint16_t*>(y.data_ptr()), ws.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "pdt_bn_fwd_eval failed");
  return y;
}

std::vector<Tensor> bn_bwd_train(Tensor dy, Tensor x, c10::optional<Tensor> mask, c10::optional<Tensor> weight,
                                 Tensor mean, Tensor invstd, bool relu, bool has_res, bool need_dgamma) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides(), "pdt bn bwd: dy layout mismatch");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 64 == 0, "pdt bn bwd: C must be a multiple of 64");
  auto dx = at::empty_like(x);
  Tensor dres;
  if (has_res) dres = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  Tensor dg, db;
  if (need_dgamma) {
    dg = at::empty({C}, fopt);
    db = at::empty({C}, fopt);
  }
  auto ws = at::empty({bn_ws_floats(M, C)}, fopt);
  const uint8_t* mp = nullptr;
  if (relu) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->numel() == M * C / 8, "pdt bn bwd: relu needs the mask");
    mp = mask->data_ptr<uint8_t>();
  }
  int rc = pdt_bn_bwd_train(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                            mp, opt_fptr(weight), mean.data_ptr<float>(), invstd.data_ptr<float>(), M, (int)C, relu,
                            has_res, reinterpret_cast<uint16_t*>(dx.data_ptr()),
                            has_res ? reinterpret_cast<uint16_t*>(dres.data_ptr()) : nullptr,
                            need_dgamma ? dg.data_ptr<float>() : nullptr, need_dgamma ? db.data_ptr<float>() : nullptr,
                            ws.data_ptr<float>(), bn_counters(x), stream());
  TORCH_CHECK(rc == 0, "pdt_bn_bwd_train failed");
  return {dx, dres, dg, db};
}

// ResNet stem backward: max-pool gradient (the BN's dz, never returned) with the stem BatchNorm's
// backward reduction fused in, then BN finalize + apply. x: the BN input [N,64,H,W] channels_last.
// Returns {dx, dgamma, dbeta}.
std::vector<Tensor> maxpool3s2_bwd_bn(Tensor dy, Tensor code, Tensor x, c10::optional<Tensor> weight, Tensor mean,
                                      Tensor invstd, bool need_dgamma) {
  check_nhwc_bf16(dy, "dy");
  check_nhwc_bf16(x, "x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C == 64, "maxpool3s2_bwd_bn: C == 64");
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == C && dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1,
              "maxpool3s2_bwd_bn: dy shape");
  TORCH_CHECK(code.scalar_type() == at::kByte && code.numel() == dy.numel(), "maxpool3s2_bwd_bn: code");
  auto dz = at::empty_like(x);
  auto dx = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  Tensor dg, db;
  if (need_dgamma) {
    dg = at::empty({C}, fopt);
    db = at::empty({C}, fopt);
  }
  const int T = pdt_maxpool_bn_parts((int)N, (int)H);
  auto part = at::empty({2 * (int64_t)T * C}, fopt);
  auto ws = at::empty({pdt_bn_tiles_ws_floats(T, (int)C) + 2 * C}, fopt);
  const int rc = pdt_maxpool3s2_bwd_bn(reinterpret_cast<const uint16_t*>(dy.data_ptr()), code.data_ptr<uint8_t>(),
                                       reinterpret_cast<uint16_t*>(dz.data_ptr()), (int)N, (int)H, (int)W, (int)C,
                                       reinterpret_cast<const uint16_t*>(x.data_ptr()), opt_fptr(weight),
                                       mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                       reinterpret_cast<uint16_t*>(dx.data_ptr()),
                                       need_dgamma ? dg.data_ptr<float>() : nullptr,
                                       need_dgamma ? db.data_ptr<float>() : nullptr, part.data_ptr<float>(),
                                       ws.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "pdt_maxpool3s2_bwd_bn failed: ", rc);
  return {dx, dg, db};
}

// Same without the BN apply: returns {dz (the max-pool gradient = dy at the BN output), coef [3, 64]
// (A, B, D: dx = A dz + B (x - mean) + D), dgamma, dbeta} for stem_conv_wgrad_bn.
std::vector<Tensor> maxpool3s2_bwd_bn_coef(Tensor dy, Tensor code, Tensor x, c10::optional<Tensor> weight,
                                           Tensor mean, Tensor invstd, bool need_dgamma, bool write_dz) {
  check_nhwc_bf16(dy, "dy");
  check_nhwc_bf16(x, "x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C == 64, "maxpool3s2_bwd_bn_coef: C == 64");
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == C && dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1,
              "maxpool3s2_bwd_bn_coef: dy shape");
  TORCH_CHECK(code.scalar_type() == at::kByte && code.numel() == dy.numel(), "maxpool3s2_bwd_bn_coef: code");
  Tensor dz;
  if (write_dz) dz = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto coef = at::empty({3, C}, fopt);
  Tensor dg, db;
  if (need_dgamma) {
    dg = at::empty({C}, fopt);
    db = at::empty({C}, fopt);
  }
  const int T = pdt_maxpool_bn_parts((int)N, (int)H);
  auto part = at::empty({2 * (int64_t)T * C}, fopt);
  auto ws = at::empty({pdt_bn_tiles_ws_floats(T, (int)C) + 2 * C}, fopt);
  const int rc = pdt_maxpool3s2_bwd_bn_coef(
      reinterpret_cast<const uint16_t*>(dy.data_ptr()), code.data_ptr<uint8_t>(),
      write_dz ? reinterpret_cast<uint16_t*>(dz.data_ptr()) : nullptr, (int)N, (int)H, (int)W, (int)C,
      reinterpret_cast<const uint16_t*>(x.data_ptr()), opt_fptr(weight), mean.data_ptr<float>(),
      invstd.data_ptr<float>(), coef.data_ptr<float>(), need_dgamma ? dg.data_ptr<float>() : nullptr,
      need_dgamma ? db.data_ptr<float>() : nullptr, part.data_ptr<float>(), ws.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "pdt_maxpool3s2_bwd_bn_coef failed: ", rc);
  return {dz, coef, dg, db};
}

// BN training backward with the reduction taken from the dy producer's per-tile partials
// (conv1x1_gemm with bn_x): finalize + apply only.
std::vector<Tensor> bn_bwd_train_tiles(Tensor dy, Tensor x, Tensor part, c10::optional<Tensor> mask,
                                       c10::optional<Tensor> weight, Tensor mean, Tensor invstd, bool relu,
                                       bool has_res, bool need_dgamma) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides(), "pdt bn bwd: dy layout mismatch");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  const int BMt = pdt_conv1x1_tile_rows();
  // any tile count: backward partials are plain sums (stride-2 data gradient: 4 phases of tiles)
  const int64_t T = part.dim() == 3 ? part.size(1) : 0;
  TORCH_CHECK(C % 64 == 0, "pdt bn bwd: C must be a multiple of 64");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3 && part.size(0) == 2 &&
              T >= 1 && part.size(2) == C, "bn_bwd_train_tiles: partials [2, T, C] fp32 expected");
  auto dx = at::empty_like(x);
  Tensor dres;
  if (has_res) dres = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  Tensor dg, db;
  if (need_dgamma) {
    dg = at::empty({C}, fopt);
    db = at::empty({C}, fopt);
  }
  auto ws = at::empty({pdt_bn_tiles_ws_floats((int)T, (int)C) + 2 * C}, fopt);
  const uint8_t* mp = nullptr;
  if (relu) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->numel() == M * C / 8, "pdt bn bwd: relu needs the mask");
    mp = mask->data_ptr<uint8_t>();
  }
  const int rc = pdt_bn_bwd_train_tiles(part.data_ptr<float>(), (int)T, BMt, reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                        reinterpret_cast<const uint16_t*>(x.data_ptr()), mp, opt_fptr(weight),
                                        mean.data_ptr<float>(), invstd.data_ptr<float>(), M, (int)C, relu, has_res,
                                        reinterpret_cast<uint16_t*>(dx.data_ptr()),
                                        has_res ? reinterpret_cast<uint16_t*>(dres.data_ptr()) : nullptr,
                                        need_dgamma ? dg.data_ptr<float>() : nullptr,
                                        need_dgamma ? db.data_ptr<float>() : nullptr, ws.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "pdt_bn_bwd_train_tiles failed: ", rc);
  return {dx, dres, dg, db};
}

// BN training backward WITHOUT the apply: {coef [3, C] (A, B, D: dx = A dy m + B (x - mean) + D),
// dgamma, dbeta} for a consumer that forms dx while loading its operand (conv1x1_bwd_fused). The
// reduction comes from the dy producer's partials [2, T, C] when given, else from a pass over (dy, x).
std::vector<Tensor> bn_bwd_coef(Tensor dy, Tensor x, c10::optional<Tensor> part, c10::optional<Tensor> mask,
                                c10::optional<Tensor> weight, Tensor mean, Tensor invstd, bool relu, bool need_dgamma) {
  check_nhwc_bf16(x, "x");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 64 == 0, "pdt bn coef: C must be a multiple of 64");
  auto fopt = x.options().dtype(at::kFloat);
  auto coef = at::empty({3, C}, fopt);
  Tensor dg, db;
  if (need_dgamma) {
    dg = at::empty({C}, fopt);
    db = at::empty({C}, fopt);
  }
  int rc;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(part->scalar_type() == at::kFloat && part->is_contiguous() && part->dim() == 3 && part->size(0) == 2 &&
                part->size(1) >= 1 && part->size(2) == C, "bn_bwd_coef: partials [2, T, C] fp32 expected");
    const int T = (int)part->size(1);
    auto ws = at::empty({pdt_bn_tiles_ws_floats(T, (int)C)}, fopt);
    rc = pdt_bn_bwd_coef_tiles(part->data_ptr<float>(), T, opt_fptr(weight), invstd.data_ptr<float>(), M, (int)C,
                               coef.data_ptr<float>(), need_dgamma ? dg.data_ptr<float>() : nullptr,
                               need_dgamma ? db.data_ptr<float>() : nullptr, ws.data_ptr<float>(), stream());
  } else {
    TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides(), "pdt bn coef: dy layout mismatch");
    const uint8_t* mp = nullptr;
    if (relu) {
      TORCH_CHECK(mask.has_value() && mask->defined() && mask->numel() == M * C / 8, "pdt bn coef: relu needs the mask");
      mp = mask->data_ptr<uint8_t>();
    }
    auto ws = at::empty({bn_ws_floats(M, C)}, fopt);
    rc = pdt_bn_bwd_coef(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                         mp, opt_fptr(weight), mean.data_ptr<float>(), invstd.data_ptr<float>(), M, (int)C, relu,
                         coef.data_ptr<float>(), need_dgamma ? dg.data_ptr<float>() : nullptr,
                         need_dgamma ? db.data_ptr<float>() : nullptr, ws.data_ptr<float>(), bn_counters(x), stream());
  }
  TORCH_CHECK(rc == 0, "pdt bn_bwd_coef failed: ", rc);
  return {coef, dg, db};
}

// Fused backward of a bottleneck's last 1x1 conv (w [C4, CW, 1, 1]: CW -> C4) and the BatchNorm that
// follows it (csrc/kernels/conv1x1_bwd_fused.hip): from dy (gradient at that BN's output), z (its
// input), mz (its ReLU bits), mean and coef [3, C4] (A, B, D of bn_bwd_coef) and the conv input xa,
// returns {dxa, dw, part}: the conv's data and weight gradients and, when bn_x / bn_mean are given
// (xa is the output of a BatchNorm with input bn_x, ReLU bits bn_mask, batch mean bn_mean), that
// BatchNorm's backward partials [2, G, CW] (else undefined). Empty list: shape not taken.
// xcoef [2, CW] (with bn_x / bn_mean): that BatchNorm's apply was deferred to the conv's forward — xa
// (only its shape is used) is recomputed as relu(xcoef[0] bn_x + xcoef[1]), and its ReLU bits are
// computed and written into bn_mask (an output then, M*CW/8 bytes).
std::vector<Tensor> conv1x1_bwd_fused(Tensor dy, Tensor z, Tensor mz, Tensor mean, Tensor coef, Tensor w, Tensor xa,
                                      c10::optional<Tensor> bn_x, c10::optional<Tensor> bn_mask,
                                      c10::optional<Tensor> bn_mean, c10::optional<Tensor> xcoef,
                                      c10::optional<Tensor> wt_pre) {
  check_nhwc_bf16(dy, "dy");
  check_nhwc_bf16(z, "z");
  TORCH_CHECK(xa.dim() == 4 && xa.is_cuda() && xa.scalar_type() == at::kBFloat16, "conv1x1_bwd_fused: xa");
  const bool recomp = xcoef.has_value() && xcoef->defined();
  if (!recomp) check_nhwc_bf16(xa, "xa");
  const int64_t C4 = z.size(1), CW = xa.size(1);
  const int64_t M = z.numel() / C4;
  if (!pdt_conv1x1_bwd_fused_ok((int)C4, (int)CW) || M * C4 >= ((int64_t)1 << 31)) return {};
  TORCH_CHECK(dy.sizes() == z.sizes() && dy.strides() == z.strides(), "conv1x1_bwd_fused: dy / z layout mismatch");
  TORCH_CHECK(xa.numel() == M * CW, "conv1x1_bwd_fused: xa pixels");
  TORCH_CHECK(mz.scalar_type() == at::kByte && mz.numel() == M * C4 / 8 && mz.is_cuda(), "conv1x1_bwd_fused: mask");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && mean.numel() == C4 && coef.scalar_type() == at::kFloat &&
              coef.is_contiguous() && coef.numel() == 3 * C4, "conv1x1_bwd_fused: mean [C4], coef [3, C4] fp32");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.numel() == C4 * CW && w.size(0) == C4,
              "conv1x1_bwd_fused: weight [C4, CW, 1, 1] bf16");
  Tensor wt;
  if (wt_pre.has_value() && wt_pre->defined()) {  // W^T from the step's batched weight prep
    TORCH_CHECK(wt_pre->scalar_type() == at::kBFloat16 && wt_pre->is_contiguous() && wt_pre->dim() == 2 &&
                    wt_pre->size(0) == CW && wt_pre->size(1) == C4,
                "conv1x1_bwd_fused: wt [CW, C4] bf16");
    wt = *wt_pre;
  } else {
    wt = w.reshape({C4, CW}).t().contiguous();
  }
  auto dxa = at::empty({xa.size(0), CW, xa.size(2), xa.size(3)}, xa.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto dw = at::empty({C4, CW}, w.options());
  const int G = pdt_conv1x1_bwd_fused_grid((int)M, (int)C4, (int)CW);
  auto fopt = z.options().dtype(at::kFloat);
  auto ws = at::empty({(int64_t)G * C4 * CW}, fopt);
  const bool bst = bn_x.has_value() && bn_x->defined();
  Tensor part;
  const uint16_t* bx = nullptr;
  const uint8_t* bm = nullptr;
  const float* bmu = nullptr;
  if (bst) {
    check_nhwc_bf16(*bn_x, "bn_x");
    TORCH_CHECK(bn_x->numel() == M * CW && bn_mean.has_value() && bn_mean->defined() &&
                bn_mean->scalar_type() == at::kFloat && bn_mean->numel() == CW, "conv1x1_bwd_fused: bn_x / bn_mean");
    if (bn_mask.has_value() && bn_mask->defined()) {
      TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() == M * CW / 8, "conv1x1_bwd_fused: bn_mask");
      bm = bn_mask->data_ptr<uint8_t>();
    }
    bx = reinterpret_cast<const uint16_t*>(bn_x->data_ptr());
    bmu = bn_mean->data_ptr<float>();
    part = at::empty({2, G, CW}, fopt);
  }
  const float* xcp = nullptr;
  uint8_t* mout = nullptr;
  if (recomp) {
    TORCH_CHECK(bst && bm, "conv1x1_bwd_fused: xcoef needs bn_x, bn_mean and the bn_mask output");
    TORCH_CHECK(xcoef->scalar_type() == at::kFloat && xcoef->is_contiguous() && xcoef->numel() == 2 * CW,
                "conv1x1_bwd_fused: xcoef [2, CW] fp32");
    xcp = xcoef->data_ptr<float>();
    mout = bn_mask->data_ptr<uint8_t>();
    bm = nullptr;
  }
  const float* cp = coef.data_ptr<float>();
  const int rc = pdt_conv1x1_bwd_fused(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                       reinterpret_cast<const uint16_t*>(z.data_ptr()), mz.data_ptr<uint8_t>(),
                                       mean.data_ptr<float>(), cp, cp + C4, cp + 2 * C4,
                                       reinterpret_cast<const uint16_t*>(wt.data_ptr()),
                                       recomp ? nullptr : reinterpret_cast<const uint16_t*>(xa.data_ptr()), bx, bm, bmu,
                                       bst ? part.data_ptr<float>() : nullptr, xcp, mout,
                                       reinterpret_cast<uint16_t*>(dxa.data_ptr()),
                                       reinterpret_cast<uint16_t*>(dw.data_ptr()), ws.data_ptr<float>(), (int)M, (int)C4,
                                       (int)CW, stream());
  TORCH_CHECK(rc == 0, "pdt_conv1x1_bwd_fused failed: ", rc);
  return {dxa, dw.view(w.sizes()), part};
}

// ----------------------------------------------------------------------------- LeNet tail (fp32)
// The reference LeNet after the stem (cnn.py:13-22) in one forward kernel / two backward kernels
// (csrc/kernels/lenet_tail.hip). ws: the 8 tail parameters in module order (w2, b2, w3, b3, fw1, fb1,
// fw2, fb2), contiguous fp32.
void check_tail_params(const std::vector<Tensor>& w) {
  TORCH_CHECK(w.size() == 8, "lenet_tail: 8 parameters (conv2 w/b, conv3 w/b, fc1 w/b, fc2 w/b)");
  const int64_t numel[8] = {2400, 16, 48000, 120, 10080, 84, 840, 10};
  for (int i = 0; i < 8; ++i) {
    check_cuda(w[i], "lenet_tail param");
    TORCH_CHECK(w[i].scalar_type() == at::kFloat && w[i].is_contiguous() && w[i].numel() == numel[i],
                "lenet_tail: parameter ", i, " must be contiguous fp32 with ", numel[i], " elements");
  }
}

std::vector<Tensor> lenet_tail_fwd(Tensor p1, std::vector<Tensor> w, double slope) {
  check_tail_params(w);
  check_cuda(p1, "p1");
  TORCH_CHECK(p1.scalar_type() == at::kFloat && p1.is_contiguous() && p1.dim() == 4 && p1.size(1) == 6 &&
              p1.size(2) == 14 && p1.size(3) == 14, "lenet_tail_fwd: p1 [N,6,14,14] contiguous fp32");
  const int64_t N = p1.size(0);
  auto o = p1.options();
  auto logits = at::empty({N, 10}, o);
  auto code2 = at::empty({N, 400}, o.dtype(at::kByte));
  auto p2 = at::empty({N, 400}, o), h3 = at::empty({N, 120}, o), h4 = at::empty({N, 84}, o);
  const int rc = pdt_lenet_tail_fwd(p1.data_ptr<float>(), w[0].data_ptr<float>(), w[1].data_ptr<float>(),
                                    w[2].data_ptr<float>(), w[3].data_ptr<float>(), w[4].data_ptr<float>(),
                                    w[5].data_ptr<float>(), w[6].data_ptr<float>(), w[7].data_ptr<float>(),
                                    (float)slope, (int)N, logits.data_ptr<float>(), code2.data_ptr<uint8_t>(),
                                    p2.data_ptr<float>(), h3.data_ptr<float>(), h4.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "pdt_lenet_tail_fwd failed: ", rc);
  return {logits, code2, p2, h3, h4};
}

// -> {dp1, dw2, db2, dw3, db3, dfw1, dfb1, dfw2, dfb2} (parameter gradients in the parameters' shapes)
std::vector<Tensor> lenet_tail_bwd(Tensor dl, Tensor p1, std::vector<Tensor> w, double slope, Tensor code2, Tensor p2,
                                   Tensor h3, Tensor h4) {
  check_tail_params(w);
  const int64_t N = p1.size(0);
  dl = dl.contiguous().to(at::kFloat);
  TORCH_CHECK(dl.numel() == N * 10 && code2.numel() == N * 400 && p2.numel() == N * 400 && h3.numel() == N * 120 &&
              h4.numel() == N * 84, "lenet_tail_bwd: saved tensor sizes");
  auto o = p1.options();
  auto ws = at::empty({pdt_lenet_tail_ws_floats((int)N)}, o);
  auto dp1 = at::empty_like(p1);
  std::vector<Tensor> g;
  for (const auto& t : w) g.push_back(at::empty_like(t));
  const int rc = pdt_lenet_tail_bwd(dl.data_ptr<float>(), p1.data_ptr<float>(), w[0].data_ptr<float>(),
                                    w[1].data_ptr<float>(), w[2].data_ptr<float>(), w[3].data_ptr<float>(),
                                    w[4].data_ptr<float>(), w[5].data_ptr<float>(), w[6].data_ptr<float>(),
                                    w[7].data_ptr<float>(), (float)slope, (int)N, code2.data_ptr<uint8_t>(),
                                    p2.data_ptr<float>(), h3.data_ptr<float>(), h4.data_ptr<float>(),
                                    ws.data_ptr<float>(), dp1.data_ptr<float>(), g[0].data_ptr<float>(),
                                    g[1].data_ptr<float>(), g[2].data_ptr<float>(), g[3].data_ptr<float>(),
                                    g[4].data_ptr<float>(), g[5].data_ptr<float>(), g[6].data_ptr<float>(),
                                    g[7].data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "pdt_lenet_tail_bwd failed: ", rc);
  return {dp1, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7]};
}

// ----------------------------------------------------------------------------- 1x1 conv GEMM (+ BN stats)
// out[M,N] = a[M,K] @ b[N,K]^T (+ out, when acc: in-place accumulate). a, b, out: row-major bf16
// (a 1x1 conv's channels_last activations viewed as [N*H*W, C]). stats: also return the per-tile
// partials [2, T, N] fp32 (tile sums, centred tile sums of squares; T = ceil(M / 256)).
// bn_x / bn_mask / bn_mean: out is the gradient at the output of a BatchNorm with this input
// (channels_last [M, N] bf16), ReLU bit-mask (or none) and batch mean: return that BatchNorm's
// backward per-tile partials [2, T, N] fp32 (sum dz, sum dz (x - mean)) instead (not with stats).
// a_coef [2, K] fp32 (optional): a is the INPUT of a BatchNorm + ReLU whose apply is deferred to here —
// the GEMM uses relu(a_coef[0] * a + a_coef[1]) per channel (forward only; not with acc / bn_x).
c10::optional<Tensor> conv1x1_gemm(Tensor a, Tensor b, Tensor out, bool acc, bool stats,
                                   c10::optional<Tensor> c_in, c10::optional<Tensor> c_mask,
                                   c10::optional<Tensor> bn_x, c10::optional<Tensor> bn_mask,
                                   c10::optional<Tensor> bn_mean, int64_t c_stride, int64_t c_H, int64_t c_W,
                                   c10::optional<Tensor> a_coef, bool bn_sum_only, bool no_store) {
  for (const Tensor* t : {&a, &b, &out}) {
    check_cuda(*t, "conv1x1_gemm operand");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->dim() == 2 && t->is_contiguous(),
                "conv1x1_gemm: operands must be 2-D contiguous bf16");
  }
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && out.size(0) == M && out.size(1) == N, "conv1x1_gemm: shape mismatch");
  TORCH_CHECK(K % 32 == 0 && N % 64 == 0, "conv1x1_gemm: K % 32 == 0 and N % 64 == 0 required");
  TORCH_CHECK(!(acc && stats), "conv1x1_gemm: acc and stats are exclusive");
  // acc source: out itself (in place), or c_in [M, N] (then optionally masked by c_mask, M*N/8 bytes)
  const uint16_t* cp = acc ? reinterpret_cast<const uint16_t*>(out.data_ptr()) : nullptr;
  const uint8_t* mp = nullptr;
  if (c_in.has_value() && c_in->defined()) {
    TORCH_CHECK(acc, "conv1x1_gemm: c_in needs acc");
    check_cuda(*c_in, "c_in");
    // c_stride > 0: c_in is the compact [M / (c_H c_W) * Hs * Ws, N] gradient of a stride subsampling
    TORCH_CHECK(c_stride <= 0 || (c_H > 0 && c_W > 0 && M % (c_H * c_W) == 0), "conv1x1_gemm: c_H * c_W must divide M");
    TORCH_CHECK(c_stride <= 0 || !(c_mask.has_value() && c_mask->defined()), "conv1x1_gemm: c_stride excludes c_mask");
    const int64_t cm_rows = c_stride > 0 ? M / (c_H * c_W) * ((c_H - 1) / c_stride + 1) * ((c_W - 1) / c_stride + 1) : M;
    TORCH_CHECK(c_in->scalar_type() == at::kBFloat16 && c_in->numel() == cm_rows * N && c_in->is_contiguous(
                    c_in->dim() == 4 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous),
                "conv1x1_gemm: c_in must be [M, N] bf16 (channels_last when 4-D)");
    cp = reinterpret_cast<const uint16_t*>(c_in->data_ptr());
  }
  if (c_mask.has_value() && c_mask->defined()) {
    TORCH_CHECK(acc && c_mask->scalar_type() == at::kByte && c_mask->numel() == M * N / 8,
                "conv1x1_gemm: c_mask must be uint8 [M * N / 8] with acc");
    mp = c_mask->data_ptr<uint8_t>();
  }
  TORCH_CHECK(c_stride <= 0 || (c_in.has_value() && c_in->defined()), "conv1x1_gemm: c_stride needs c_in");
  c10::optional<Tensor> part;
  const int64_t T = (M + pdt_conv1x1_tile_rows() - 1) / pdt_conv1x1_tile_rows();
  if (stats) part = at::empty({2, T, N}, a.options().dtype(at::kFloat));
  // bn_sum_only: the BatchNorm input is not read; only the partials' sum(dz) row is meaningful (ALG backward)
  const bool bstats = (bn_x.has_value() && bn_x->defined()) || bn_sum_only;
  const uint16_t* bx = nullptr;
  const uint8_t* bm = nullptr;
  const float* bmean = nullptr;
  if (bstats) {
    TORCH_CHECK(!stats, "conv1x1_gemm: stats and bn_x are exclusive");
    if (!bn_sum_only) {
      check_cuda(*bn_x, "bn_x");
      TORCH_CHECK(bn_x->scalar_type() == at::kBFloat16 && bn_x->numel() == M * N && bn_x->is_contiguous(
                      bn_x->dim() == 4 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous),
                  "conv1x1_gemm: bn_x must be [M, N] bf16 (channels_last when 4-D)");
      bx = reinterpret_cast<const uint16_t*>(bn_x->data_ptr());
    }
    TORCH_CHECK(bn_mean.has_value() && bn_mean->defined() && bn_mean->scalar_type() == at::kFloat &&
                bn_mean->numel() == N && bn_mean->is_contiguous() && bn_mean->is_cuda(),
                "conv1x1_gemm: bn_mean must be fp32 [N]");
    if (bn_mask.has_value() && bn_mask->defined()) {
      TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() == M * N / 8 && bn_mask->is_cuda(),
                  "conv1x1_gemm: bn_mask must be uint8 [M * N / 8]");
      bm = bn_mask->data_ptr<uint8_t>();
    }
    bmean = bn_mean->data_ptr<float>();
    part = at::empty({2, T, N}, a.options().dtype(at::kFloat));
  }
  const float* acp = nullptr;
  if (a_coef.has_value() && a_coef->defined()) {
    TORCH_CHECK(!acc && !bstats, "conv1x1_gemm: a_coef is forward-only (no acc / bn_x)");
    TORCH_CHECK(a_coef->scalar_type() == at::kFloat && a_coef->is_contiguous() && a_coef->numel() == 2 * K &&
                a_coef->is_cuda(), "conv1x1_gemm: a_coef must be fp32 [2, K]");
    acp = a_coef->data_ptr<float>();
  }
  const int rc = pdt_conv1x1_gemm(reinterpret_cast<const uint16_t*>(a.data_ptr()),
                                  reinterpret_cast<const uint16_t*>(b.data_ptr()),
                                  reinterpret_cast<uint16_t*>(out.data_ptr()), cp, mp,
                                  stats ? part->data_ptr<float>() : nullptr, (int)M, (int)K, (int)N, bx, bm, bmean,
                                  bstats ? part->data_ptr<float>() : nullptr, (int)c_stride, (int)c_H, (int)c_W, acp,
                                  stream(), no_store ? 1 : 0);
  TORCH_CHECK(rc == 0, "pdt_conv1x1_gemm failed: ", rc);
  return part;
}

// A BatchNorm (+ residual) + ReLU applied in the epilogue of the 1x1-conv GEMM that produced its input
// (csrc/kernels/conv1x1.hip APPLY): y = relu(ab[0] * (a b^T) + ab[1] + r), r = res or rab[0] res + rab[1].
// a [M, K], b [N, K] bf16 row-major; res: the residual (bf16, M * N elements, channels_last when 4-D; y gets
// its shape / layout); ab, rab: fp32 [2, N]; a_coef: fp32 [2, K] (A is a deferred BatchNorm input, ATR).
// Returns {y, mask uint8 [M * N / 8]}.
std::vector<Tensor> conv1x1_gemm_apply(Tensor a, Tensor b, Tensor res, Tensor ab, c10::optional<Tensor> rab,
                                       c10::optional<Tensor> a_coef) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  check_cuda(res, "res");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1) && a.scalar_type() == at::kBFloat16 &&
                  b.scalar_type() == at::kBFloat16 && a.is_contiguous() && b.is_contiguous(),
              "conv1x1_gemm_apply: a [M, K], b [N, K] contiguous bf16");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  const auto fmt = res.dim() == 4 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
  TORCH_CHECK(res.scalar_type() == at::kBFloat16 && res.numel() == M * N && res.is_contiguous(fmt) &&
                  (res.dim() != 4 || res.size(1) == N),
              "conv1x1_gemm_apply: res must be [M, N] bf16 (channels_last when 4-D)");
  auto f32 = [&](const Tensor& t, int64_t n, const char* what) {
    check_cuda(t, what);
    TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n, "conv1x1_gemm_apply: ", what,
                " must be fp32 contiguous with ", n, " elements");
    return t.data_ptr<float>();
  };
  const float* abp = f32(ab, 2 * N, "ab");
  const float* rabp = (rab.has_value() && rab->defined()) ? f32(*rab, 2 * N, "rab") : nullptr;
  const float* acp = (a_coef.has_value() && a_coef->defined()) ? f32(*a_coef, 2 * K, "a_coef") : nullptr;
  auto y = at::empty_like(res, res.options(), fmt);
  auto mask = at::empty({M * N / 8}, res.options().dtype(at::kByte));
  const int rc = pdt_conv1x1_gemm_apply(reinterpret_cast<const uint16_t*>(a.data_ptr()),
                                        reinterpret_cast<const uint16_t*>(b.data_ptr()),
                                        reinterpret_cast<uint16_t*>(y.data_ptr()),
                                        reinterpret_cast<const uint16_t*>(res.data_ptr()), abp, rabp,
                                        mask.data_ptr<uint8_t>(), (int)M, (int)K, (int)N, acp, stream());
  TORCH_CHECK(rc == 0, "pdt_conv1x1_gemm_apply failed: ", rc);
  return {y, mask};
}

// Batched per-step weight transforms (csrc/kernels/weight_prep.hip): for each i, src[i] = a conv weight
// [Co, Ci, k, k] bf16 (k = 1: any layout; k = 3: channels_last, storage [Co][3][3][Ci]) -> dst[i]: k = 1:
// W^T [Ci, Co] contiguous; k = 3: the flipped transposed weights [Ci, Co, 3, 3] channels_last (= conv3x3_flip).
void weight_prep(std::vector<Tensor> src, std::vector<Tensor> dst) {
  TORCH_CHECK(src.size() == dst.size(), "weight_prep: src / dst lists differ");
  const int cap = pdt_weight_prep_max_items();
  std::vector<const uint16_t*> sp;
  std::vector<uint16_t*> dp;
  std::vector<int> R, C, T;
  auto flush = [&]() {
    if (sp.empty()) return;
    TORCH_CHECK(pdt_weight_prep(sp.data(), dp.data(), R.data(), C.data(), T.data(), (int)sp.size(), stream()) == 0,
                "pdt_weight_prep failed");
    sp.clear(); dp.clear(); R.clear(); C.clear(); T.clear();
  };
  for (size_t i = 0; i < src.size(); ++i) {
    const Tensor& w = src[i];
    const Tensor& d = dst[i];
    check_cuda(w, "src");
    check_cuda(d, "dst");
    TORCH_CHECK(w.dim() == 4 && w.scalar_type() == at::kBFloat16 && d.scalar_type() == at::kBFloat16 &&
                    w.size(2) == w.size(3) && (w.size(2) == 1 || w.size(2) == 3),
                "weight_prep: bf16 [Co, Ci, k, k] weights, k = 1 or 3");
    const int64_t Co = w.size(0), Ci = w.size(1), k = w.size(2);
    if (k == 1) {
      TORCH_CHECK(w.is_contiguous() || w.is_contiguous(at::MemoryFormat::ChannelsLast), "weight_prep: 1x1 weight layout");
      TORCH_CHECK(d.dim() == 2 && d.size(0) == Ci && d.size(1) == Co && d.is_contiguous(), "weight_prep: dst [Ci, Co]");
    } else {
      TORCH_CHECK(w.is_contiguous(at::MemoryFormat::ChannelsLast), "weight_prep: 3x3 weight must be channels_last");
      TORCH_CHECK(d.dim() == 4 && d.size(0) == Ci && d.size(1) == Co && d.size(2) == 3 && d.size(3) == 3 &&
                      d.is_contiguous(at::MemoryFormat::ChannelsLast),
                  "weight_prep: dst [Ci, Co, 3, 3] channels_last");
    }
    sp.push_back(reinterpret_cast<const uint16_t*>(w.data_ptr()));
    dp.push_back(reinterpret_cast<uint16_t*>(d.data_ptr()));
    R.push_back((int)Co);
    C.push_back((int)Ci);
    T.push_back((int)(k * k));
    if ((int)sp.size() == cap) flush();
  }
  flush();
}

// Weight gradient of a stride-1 1x1 conv (csrc/kernels/conv1x1_wgrad.hip): dw [Co, Ci] bf16 =
// dy[M, Co]^T x[M, Ci] from the row-major bf16 NHWC views (split-K over pixels, fixed-order fp32
// reduction). Returns an undefined tensor for a shape the kernel does not take (caller falls back).
Tensor conv1x1_wgrad(Tensor x, Tensor dy) {
  check_cuda(x, "x");
  check_cuda(dy, "dy");
  TORCH_CHECK(x.dim() == 2 && dy.dim() == 2 && x.size(0) == dy.size(0), "conv1x1_wgrad: x [M, Ci], dy [M, Co]");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16 && x.is_contiguous() &&
                  dy.is_contiguous(),
              "conv1x1_wgrad: contiguous bf16 operands");
  const int64_t M = x.size(0), Ci = x.size(1), Co = dy.size(1);
  if (M * std::max(Ci, Co) >= ((int64_t)1 << 31)) return Tensor();
  int ns = 0;
  const int64_t wsf = pdt_conv1x1_wgrad_ws_floats((int)M, (int)Ci, (int)Co, &ns);
  if (wsf == 0) return Tensor();
  auto ws = at::empty({wsf}, x.options().dtype(at::kFloat));
  auto dw = at::empty({Co, Ci}, x.options());
  const int rc = pdt_conv1x1_wgrad(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                   reinterpret_cast<uint16_t*>(dw.data_ptr()), ws.data_ptr<float>(), (int)M, (int)Ci,
                                   (int)Co, stream());
  if (rc == -1 || rc == -2) return Tensor();
  TORCH_CHECK(rc == 0, "pdt_conv1x1_wgrad failed: ", rc);
  return dw;
}

// ALG backward of conv3 + bn3 (csrc/kernels/bn_alg.hip, ops/conv.py _bwd_alg): [dy1 | dy2 | 1]^T x in fp32,
// rows co1 + co2 (+ the ones block: column sums of x). x [M, Ci], dy1 [M, co1], dy2 [M, co2] contiguous bf16.
// Returns an empty tensor for an unsupported shape.
Tensor conv1x1_wgrad_seg(Tensor x, Tensor dy1, Tensor dy2) {
  for (const Tensor* t : {&x, &dy1, &dy2}) {
    check_cuda(*t, "conv1x1_wgrad_seg operand");
    TORCH_CHECK(t->dim() == 2 && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->size(0) == x.size(0),
                "conv1x1_wgrad_seg: contiguous bf16 [M, *] operands");
  }
  const int64_t M = x.size(0), Ci = x.size(1), co1 = dy1.size(1), co2 = dy2.size(1);
  if (M * std::max(std::max(Ci, co1), co2) >= ((int64_t)1 << 31)) return Tensor();
  int rows = 0;
  const int64_t wsf = pdt_conv1x1_wgrad_seg_ws_floats((int)M, (int)Ci, (int)co1, (int)co2, &rows);
  if (wsf == 0) return Tensor();
  auto ws = at::empty({wsf}, x.options().dtype(at::kFloat));
  auto out = at::empty({rows, Ci}, x.options().dtype(at::kFloat));
  const int rc = pdt_conv1x1_wgrad_seg(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                       reinterpret_cast<const uint16_t*>(dy1.data_ptr()), (int)co1,
                                       reinterpret_cast<const uint16_t*>(dy2.data_ptr()), (int)co2, out.data_ptr<float>(),
                                       ws.data_ptr<float>(), (int)M, (int)Ci, stream());
  if (rc == -1 || rc == -2) return Tensor();
  TORCH_CHECK(rc == 0, "pdt_conv1x1_wgrad_seg failed: ", rc);
  return out;
}

// out[M, N] = [a1 | a2 x rep2 | 1] b^T (b [N, k1 + rep2 k2 + 32]) with the BSTATS epilogue when bn_x is given
// (then returns the backward partials [2, T, N], as conv1x1_gemm).
c10::optional<Tensor> conv1x1_gemm_seg(Tensor a1, Tensor a2, int64_t rep2, Tensor b, Tensor out,
                                       c10::optional<Tensor> bn_x, c10::optional<Tensor> bn_mask,
                                       c10::optional<Tensor> bn_mean) {
  for (const Tensor* t : {&a1, &a2, &b, &out}) {
    check_cuda(*t, "conv1x1_gemm_seg operand");
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->dim() == 2 && t->is_contiguous(),
                "conv1x1_gemm_seg: operands must be 2-D contiguous bf16");
  }
  const int64_t M = a1.size(0), k1 = a1.size(1), k2 = a2.size(1), N = b.size(0);
  TORCH_CHECK(a2.size(0) == M && out.size(0) == M && out.size(1) == N && b.size(1) == k1 + rep2 * k2 + 32 && rep2 >= 1,
              "conv1x1_gemm_seg: shape mismatch");
  TORCH_CHECK(k1 % 32 == 0 && k2 % 32 == 0 && N % 64 == 0, "conv1x1_gemm_seg: k1, k2 % 32 and N % 64 required");
  c10::optional<Tensor> part;
  const uint16_t* bx = nullptr;
  const uint8_t* bm = nullptr;
  const float* bmean = nullptr;
  if (bn_x.has_value() && bn_x->defined()) {
    check_cuda(*bn_x, "bn_x");
    TORCH_CHECK(bn_x->scalar_type() == at::kBFloat16 && bn_x->numel() == M * N && bn_x->is_contiguous(
                    bn_x->dim() == 4 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous),
                "conv1x1_gemm_seg: bn_x must be [M, N] bf16 (channels_last when 4-D)");
    TORCH_CHECK(bn_mean.has_value() && bn_mean->defined() && bn_mean->scalar_type() == at::kFloat &&
                bn_mean->numel() == N && bn_mean->is_contiguous() && bn_mean->is_cuda(),
                "conv1x1_gemm_seg: bn_mean must be fp32 [N]");
    if (bn_mask.has_value() && bn_mask->defined()) {
      TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() == M * N / 8 && bn_mask->is_cuda(),
                  "conv1x1_gemm_seg: bn_mask must be uint8 [M * N / 8]");
      bm = bn_mask->data_ptr<uint8_t>();
    }
    bx = reinterpret_cast<const uint16_t*>(bn_x->data_ptr());
    bmean = bn_mean->data_ptr<float>();
    const int64_t T = (M + pdt_conv1x1_tile_rows() - 1) / pdt_conv1x1_tile_rows();
    part = at::empty({2, T, N}, a1.options().dtype(at::kFloat));
  }
  const int rc = pdt_conv1x1_gemm_seg(reinterpret_cast<const uint16_t*>(a1.data_ptr()), (int)k1,
                                      reinterpret_cast<const uint16_t*>(a2.data_ptr()), (int)k2, (int)rep2,
                                      reinterpret_cast<const uint16_t*>(b.data_ptr()),
                                      reinterpret_cast<uint16_t*>(out.data_ptr()), (int)M, (int)N, bx, bm, bmean,
                                      part.has_value() ? part->data_ptr<float>() : nullptr, stream());
  TORCH_CHECK(rc == 0, "pdt_conv1x1_gemm_seg failed: ", rc);
  return part;
}

// (bcat [CW, C4 + 2 CW + 32] bf16, dW [C4, CW] bf16) of the ALG backward (csrc/kernels/bn_alg.hip).
std::vector<Tensor> bn_alg_assemble(Tensor w, Tensor coef, Tensor mean, Tensor G, Tensor wg, Tensor BWG, int64_t rep) {
  for (const Tensor* t : {&w, &coef, &mean, &G, &wg, &BWG}) {
    check_cuda(*t, "bn_alg_assemble operand");
    TORCH_CHECK(t->is_contiguous(), "bn_alg_assemble: contiguous operands");
  }
  TORCH_CHECK(w.dim() == 2 && w.scalar_type() == at::kBFloat16, "bn_alg_assemble: w [C4, CW] bf16");
  const int64_t C4 = w.size(0), CW = w.size(1);
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.numel() == 3 * C4 && mean.scalar_type() == at::kFloat &&
                  mean.numel() == C4 && G.scalar_type() == at::kFloat && G.numel() == (C4 / 128) * CW * CW &&
                  BWG.scalar_type() == at::kFloat && BWG.numel() == std::max<int64_t>(1, CW / 128) * C4 * CW &&
                  wg.scalar_type() == at::kFloat &&
                  wg.dim() == 2 && wg.size(1) == CW && wg.size(0) > C4 + CW,
              "bn_alg_assemble: operand shapes");
  TORCH_CHECK(rep == 1 || rep == 2, "bn_alg_assemble: rep 1 or 2");
  auto bcat = at::empty({CW, C4 + rep * CW + 32}, w.options());
  auto dW = at::empty({C4, CW}, w.options());
  const int rc = pdt_bn_alg_assemble(reinterpret_cast<const uint16_t*>(w.data_ptr()), coef.data_ptr<float>(),
                                     mean.data_ptr<float>(), G.data_ptr<float>(), wg.data_ptr<float>(),
                                     BWG.data_ptr<float>(), reinterpret_cast<uint16_t*>(bcat.data_ptr()),
                                     reinterpret_cast<uint16_t*>(dW.data_ptr()), (int)C4, (int)CW, (int)rep, stream());
  TORCH_CHECK(rc == 0, "pdt_bn_alg_assemble failed: ", rc);
  return {bcat, dW};
}

// (G [CW, CW], BWG [C4, CW]) fp32 of the ALG backward: W^T diag(B) W and diag(B) W Gram (csrc/kernels/bn_alg.hip).
std::vector<Tensor> bn_alg_small_gemm(Tensor w, Tensor coef, Tensor wg, c10::optional<Tensor> wt) {
  check_cuda(w, "w");
  check_cuda(coef, "coef");
  check_cuda(wg, "wg");
  TORCH_CHECK(w.dim() == 2 && w.scalar_type() == at::kBFloat16 && w.is_contiguous(), "bn_alg_small_gemm: w [C4, CW] bf16");
  const int64_t C4 = w.size(0), CW = w.size(1);
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == 3 * C4 &&
                  wg.scalar_type() == at::kFloat && wg.is_contiguous() && wg.dim() == 2 && wg.size(1) == CW &&
                  wg.size(0) >= C4 + CW && C4 % 64 == 0 && CW % 64 == 0,
              "bn_alg_small_gemm: coef [3, C4], wg [>= C4 + CW, CW] fp32, C4 / CW % 64");
  TORCH_CHECK(C4 % 128 == 0 && (CW == 64 || CW % 128 == 0), "bn_alg_small_gemm: C4 % 128, CW 64 or % 128");
  // split-K slices (summed by bn_alg_assemble): G [C4 / 128, CW, CW], BWG [max(1, CW / 128), C4, CW]
  auto G = at::empty({C4 / 128, CW, CW}, wg.options());
  auto BWG = at::empty({std::max<int64_t>(1, CW / 128), C4, CW}, wg.options());
  const uint16_t* wtp = nullptr;
  if (wt.has_value() && wt->defined()) {  // W^T [CW, C4]: the matrix-core form
    check_cuda(*wt, "wt");
    TORCH_CHECK(wt->scalar_type() == at::kBFloat16 && wt->is_contiguous() && wt->dim() == 2 && wt->size(0) == CW &&
                    wt->size(1) == C4, "bn_alg_small_gemm: wt [CW, C4] bf16 contiguous");
    wtp = reinterpret_cast<const uint16_t*>(wt->data_ptr());
  }
  TORCH_CHECK(pdt_bn_alg_small_gemm(reinterpret_cast<const uint16_t*>(w.data_ptr()), wtp, coef.data_ptr<float>(),
                                    wg.data_ptr<float>(), G.data_ptr<float>(), BWG.data_ptr<float>(), (int)C4, (int)CW,
                                    stream()) == 0,
              "pdt_bn_alg_small_gemm failed");
  return {G, BWG};
}

// Completes a sum-only producer's BatchNorm backward partials in place (csrc/kernels/bn_alg.hip).
void bn_alg_fix_s2(Tensor part, Tensor wg, Tensor w) {
  check_cuda(part, "part");
  check_cuda(wg, "wg");
  check_cuda(w, "w");
  TORCH_CHECK(w.dim() == 2 && w.scalar_type() == at::kBFloat16 && w.is_contiguous(), "bn_alg_fix_s2: w [C4, CW] bf16");
  const int64_t C4 = w.size(0), CW = w.size(1);
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3 && part.size(0) == 2 &&
                  part.size(2) == C4 && wg.scalar_type() == at::kFloat && wg.is_contiguous() && wg.dim() == 2 &&
                  wg.size(1) == CW && wg.size(0) >= C4,
              "bn_alg_fix_s2: part [2, T, C4], wg [>= C4, CW] fp32");
  TORCH_CHECK(pdt_bn_alg_fix_s2(part.data_ptr<float>(), (int)part.size(1), wg.data_ptr<float>(),
                                reinterpret_cast<const uint16_t*>(w.data_ptr()), (int)C4, (int)CW, stream()) == 0,
              "pdt_bn_alg_fix_s2 failed");
}

// A downsample BatchNorm's backward partials [2, 1, C4] from s1 = sum(g), its mean and the ALG pass (bn_alg.hip).
Tensor bn_alg_ds_part(Tensor s1, Tensor mean, Tensor wg, Tensor w) {
  for (const Tensor* t : {&s1, &mean, &wg, &w}) check_cuda(*t, "bn_alg_ds_part operand");
  TORCH_CHECK(w.dim() == 2 && w.scalar_type() == at::kBFloat16 && w.is_contiguous(), "bn_alg_ds_part: w [C4, CW] bf16");
  const int64_t C4 = w.size(0), CW = w.size(1);
  TORCH_CHECK(s1.scalar_type() == at::kFloat && s1.is_contiguous() && s1.numel() == C4 && mean.scalar_type() == at::kFloat &&
                  mean.is_contiguous() && mean.numel() == C4 && wg.scalar_type() == at::kFloat && wg.is_contiguous() &&
                  wg.dim() == 2 && wg.size(1) == CW && wg.size(0) >= C4,
              "bn_alg_ds_part: s1 / mean [C4] fp32, wg [>= C4, CW] fp32");
  auto part = at::empty({2, 1, C4}, s1.options());
  TORCH_CHECK(pdt_bn_alg_ds_part(part.data_ptr<float>(), s1.data_ptr<float>(), mean.data_ptr<float>(),
                                 wg.data_ptr<float>(), reinterpret_cast<const uint16_t*>(w.data_ptr()), (int)C4, (int)CW,
                                 stream()) == 0,
              "pdt_bn_alg_ds_part failed");
  return part;
}

// BN training forward with the statistics taken from conv1x1_gemm's per-tile partials.
std::vector<Tensor> bn_fwd_train_tiles(Tensor x, Tensor part, c10::optional<Tensor> res, c10::optional<Tensor> weight,
                                       c10::optional<Tensor> bias, c10::optional<Tensor> running_mean,
                                       c10::optional<Tensor> running_var, double momentum, double eps, bool relu,
                                       c10::optional<Tensor> res_ab, bool apply, int64_t sub) {
  check_nhwc_bf16(x, "x");
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 64 == 0, "pdt bn: C must be a multiple of 64");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3 && part.size(0) == 2 &&
              part.size(2) == C, "bn_fwd_train_tiles: partials [2, T, C] fp32 expected");
  // tile height from the partials' row count: 256 (every producer) or 224 (the layer-1 row-tile 3x3,
  // used only where M / 224 >= 256, so the two never give the same T)
  const int64_t T = part.size(1);
  const int BMt = T == (M + 255) / 256 ? 256 : (M % 224 == 0 && T == M / 224 ? 224 : 0);
  TORCH_CHECK(BMt > 0, "bn_fwd_train_tiles: partials row count ", T, " matches no tile height for M = ", M);
  const auto rab = res_ab_ptrs(res_ab, C);
  Tensor y;
  if (apply) y = at::empty_like(x);
  Tensor mask;
  if (relu && apply) mask = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  auto ws = at::empty({pdt_bn_tiles_ws_floats((int)T, (int)C)}, fopt);
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_nhwc_bf16(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes() && res->strides() == x.strides(), "pdt bn: residual layout mismatch");
    rp = reinterpret_cast<const uint16_t*>(res->data_ptr());
  }
  float* rm = running_mean.has_value() && running_mean->defined() ? running_mean->data_ptr<float>() : nullptr;
  float* rv = running_var.has_value() && running_var->defined() ? running_var->data_ptr<float>() : nullptr;
  // sub >= 2: also the stride-sub subsample of y (x must be 4-D [N, C, H, W])
  Tensor ys;
  if (sub >= 2) {
    TORCH_CHECK(apply && x.dim() == 4, "bn_fwd_train_tiles: the subsample output needs the apply and a 4-D x");
    ys = at::empty({x.size(0), C, (x.size(2) - 1) / sub + 1, (x.size(3) - 1) / sub + 1},
                   x.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  const int rc = pdt_bn_fwd_train_tiles(part.data_ptr<float>(), (int)T, BMt, reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                        rp, rab.first, rab.second, opt_fptr(weight), opt_fptr(bias), rm, rv,
                                        (float)momentum, (float)eps, M, (int)C, relu,
                                        apply ? reinterpret_cast<uint16_t*>(y.data_ptr()) : nullptr,
                                        (relu && apply) ? mask.data_ptr<uint8_t>() : nullptr, mean.data_ptr<float>(),
                                        invstd.data_ptr<float>(), ws.data_ptr<float>(), stream(),
                                        sub >= 2 ? reinterpret_cast<uint16_t*>(ys.data_ptr()) : nullptr,
                                        sub >= 2 ? (int)x.size(2) : 0, sub >= 2 ? (int)x.size(3) : 0, (int)sub);
  if (rc == -4) return {};  // (subsample not taken: the caller gathers)
  TORCH_CHECK(rc == 0, "pdt_bn_fwd_train_tiles failed: ", rc);
  if (!apply)  // the apply coefficients (a, b) are the workspace's last 2C floats (past the level-1 sums)
    return {Tensor(), Tensor(), mean, invstd, ws.narrow(0, ws.numel() - 2 * C, 2 * C).view({2, C})};
  if (sub >= 2) return {y, mask, mean, invstd, ys};
  return {y, mask, mean, invstd};
}

// ----------------------------------------------------------------------------- 3x3 conv (stride 1, pad 1)
// y = conv2d(x, w, stride=1, padding=1) for channels_last bf16 x [N,Ci,H,W] and w [Co,Ci,3,3]
// (w's channels_last storage is [Co][3][3][Ci], the kernel's layout).
Tensor conv3x3s1_fwd(Tensor x, Tensor w) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(1) == x.size(1) &&
              w.scalar_type() == at::kBFloat16, "conv3x3: weight [Co, Ci, 3, 3] bf16");
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3), Co = w.size(0);
  auto y = at::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = pdt_conv3x3s1_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                   reinterpret_cast<uint16_t*>(y.data_ptr()), (int)N, (int)H, (int)W, (int)Ci, (int)Co,
                                   stream());
  TORCH_CHECK(rc == 0, "pdt_conv3x3s1_fwd failed: ", rc);
  return y;
}

// conv3x3s1_fwd + the per-tile BatchNorm statistics of y (tile_stats.h): {y, part [2, T, Co]}, or
// {y} alone when the shape runs on a kernel without the statistics epilogue.
std::vector<Tensor> conv3x3s1_fwd_stats(Tensor x, Tensor w) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(1) == x.size(1) &&
              w.scalar_type() == at::kBFloat16, "conv3x3: weight [Co, Ci, 3, 3] bf16");
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3), Co = w.size(0);
  auto y = at::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t rows = pdt_conv3x3s1_stats_tile_rows((int)N, (int)H, (int)W, (int)Ci, (int)Co);
  const int64_t T = (N * H * W + rows - 1) / rows;
  auto part = at::empty({2, T, Co}, x.options().dtype(at::kFloat));
  const int rc = pdt_conv3x3s1_fwd_stats(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                         reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                         reinterpret_cast<uint16_t*>(y.data_ptr()), part.data_ptr<float>(), (int)N,
                                         (int)H, (int)W, (int)Ci, (int)Co, stream());
  if (rc == -5) return {conv3x3s1_fwd(x, w)};
  TORCH_CHECK(rc == 0, "pdt_conv3x3s1_fwd_stats failed: ", rc);
  return {y, part};
}

// y = conv3x3s1(x, w) where y is the gradient at a BatchNorm's output (bn_x: that BN's input, same
// shape as y; bn_mask: its ReLU bit-mask or none; bn_mean: its batch mean): returns {y, partials
// [2, T, Co]} of the BN's backward reduction, or {y} where only a kernel without the epilogue applies.
std::vector<Tensor> conv3x3s1_fwd_bnbwd(Tensor x, Tensor w, Tensor bn_x, c10::optional<Tensor> bn_mask,
                                        Tensor bn_mean) {
  check_nhwc_bf16(x, "x");
  check_nhwc_bf16(bn_x, "bn_x");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(1) == x.size(1) &&
              w.scalar_type() == at::kBFloat16, "conv3x3: weight [Co, Ci, 3, 3] bf16");
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3), Co = w.size(0);
  TORCH_CHECK(bn_x.size(0) == N && bn_x.size(1) == Co && bn_x.size(2) == H && bn_x.size(3) == W,
              "conv3x3s1_fwd_bnbwd: bn_x must have the output's shape");
  TORCH_CHECK(bn_mean.scalar_type() == at::kFloat && bn_mean.numel() == Co && bn_mean.is_contiguous() &&
              bn_mean.is_cuda(), "conv3x3s1_fwd_bnbwd: bn_mean fp32 [Co]");
  const uint8_t* mp = nullptr;
  if (bn_mask.has_value() && bn_mask->defined()) {
    TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() == N * H * W * Co / 8 && bn_mask->is_cuda(),
                "conv3x3s1_fwd_bnbwd: bn_mask uint8 [M * Co / 8]");
    mp = bn_mask->data_ptr<uint8_t>();
  }
  auto y = at::empty({N, Co, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int64_t rows = pdt_conv3x3s1_bnbwd_tile_rows((int)N, (int)H, (int)W, (int)Ci, (int)Co);
  const int64_t T = (N * H * W + rows - 1) / rows;
  auto part = at::empty({2, T, Co}, x.options().dtype(at::kFloat));
  const int rc = pdt_conv3x3s1_fwd_bnbwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                         reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                         reinterpret_cast<uint16_t*>(y.data_ptr()),
                                         reinterpret_cast<const uint16_t*>(bn_x.data_ptr()), mp,
                                         bn_mean.data_ptr<float>(), part.data_ptr<float>(), (int)N, (int)H, (int)W,
                                         (int)Ci, (int)Co, stream());
  if (rc == -5) return {conv3x3s1_fwd(x, w)};
  TORCH_CHECK(rc == 0, "pdt_conv3x3s1_fwd_bnbwd failed: ", rc);
  return {y, part};
}

// ----------------------------------------------------------------------------- 3x3 conv (stride 2, pad 1)
// y = conv2d(x, w, stride=2, padding=1), channels_last bf16 (csrc/kernels/conv3x3_s2.hip); stats: also
// the per-tile BatchNorm statistics of y -> {y, part [2, T, Co]}. Ci % 64, Co % 128 == 0 (returns {} for
// a shape the kernel does not take).
std::vector<Tensor> conv3x3s2_fwd(Tensor x, Tensor w, bool stats) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(1) == x.size(1) &&
              w.scalar_type() == at::kBFloat16, "conv3x3s2: weight [Co, Ci, 3, 3] bf16");
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3), Co = w.size(0);
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  auto y = at::empty({N, Co, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor part;
  if (stats) part = at::empty({2, (N * Ho * Wo + 255) / 256, Co}, x.options().dtype(at::kFloat));
  const int rc = pdt_conv3x3s2_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                   reinterpret_cast<uint16_t*>(y.data_ptr()), stats ? part.data_ptr<float>() : nullptr,
                                   (int)N, (int)H, (int)W, (int)Ci, (int)Co, stream());
  if (rc == -1 || rc == -2) return {};
  TORCH_CHECK(rc == 0, "pdt_conv3x3s2_fwd failed: ", rc);
  if (stats) return {y, part};
  return {y};
}

// dx [N, Ci, H, W] of that conv from dy [N, Co, Ho, Wo] and wf = conv3x3_flip(w). With bn_x / bn_mean
// (bn_mask optional): dx is the gradient at a BatchNorm's output -> {dx, partials [2, T, Ci]} of its
// backward reduction (T = 4 phases of tiles). Returns {} for a shape the kernel does not take.
std::vector<Tensor> conv3x3s2_dgrad(Tensor dy, Tensor wf, int64_t H, int64_t W, c10::optional<Tensor> bn_x,
                                    c10::optional<Tensor> bn_mask, c10::optional<Tensor> bn_mean) {
  check_nhwc_bf16(dy, "dy");
  TORCH_CHECK(wf.dim() == 4 && wf.size(2) == 3 && wf.size(3) == 3 && wf.size(1) == dy.size(1) &&
              wf.scalar_type() == at::kBFloat16, "conv3x3s2_dgrad: flipped weight [Ci, Co, 3, 3] bf16");
  wf = wf.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = dy.size(0), Co = dy.size(1), Ci = wf.size(0);
  TORCH_CHECK(dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1, "conv3x3s2_dgrad: dy spatial size");
  auto dx = at::empty({N, Ci, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool bst = bn_x.has_value() && bn_x->defined();
  const uint16_t* bx = nullptr;
  const uint8_t* bm = nullptr;
  const float* bmean = nullptr;
  Tensor part;
  if (bst) {
    check_nhwc_bf16(*bn_x, "bn_x");
    TORCH_CHECK(bn_x->sizes() == dx.sizes(), "conv3x3s2_dgrad: bn_x must have dx's shape");
    TORCH_CHECK(bn_mean.has_value() && bn_mean->defined() && bn_mean->scalar_type() == at::kFloat &&
                bn_mean->numel() == Ci && bn_mean->is_contiguous() && bn_mean->is_cuda(),
                "conv3x3s2_dgrad: bn_mean fp32 [Ci]");
    if (bn_mask.has_value() && bn_mask->defined()) {
      TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() == N * H * W * Ci / 8 && bn_mask->is_cuda(),
                  "conv3x3s2_dgrad: bn_mask uint8 [M * Ci / 8]");
      bm = bn_mask->data_ptr<uint8_t>();
    }
    bx = reinterpret_cast<const uint16_t*>(bn_x->data_ptr());
    bmean = bn_mean->data_ptr<float>();
    part = at::empty({2, (int64_t)pdt_conv3x3s2_dgrad_tiles((int)N, (int)H, (int)W), Ci},
                     dy.options().dtype(at::kFloat));
  }
  const int rc = pdt_conv3x3s2_dgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                     reinterpret_cast<const uint16_t*>(wf.data_ptr()),
                                     reinterpret_cast<uint16_t*>(dx.data_ptr()), bx, bm, bmean,
                                     bst ? part.data_ptr<float>() : nullptr, (int)N, (int)H, (int)W, (int)Ci, (int)Co,
                                     stream());
  if (rc == -1 || rc == -2) return {};
  TORCH_CHECK(rc == 0, "pdt_conv3x3s2_dgrad failed: ", rc);
  if (bst) return {dx, part};
  return {dx};
}

// Weight gradient of the stride-2 pad-1 3x3 conv (conv3x3_wgrad.hip, S = 2): dw [Co, Ci, 3, 3]
// channels_last bf16 from x [N, Ci, H, W] and dy [N, Co, Ho, Wo]; undefined for an unsupported shape.
Tensor conv3x3s2_wgrad(Tensor x, Tensor dy) {
  check_nhwc_bf16(x, "x");
  check_nhwc_bf16(dy, "dy");
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3), Co = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1,
              "conv3x3s2_wgrad: dy [N, Co, Ho, Wo]");
  int ns = 0;
  const int64_t wsf = pdt_conv3x3s2_wgrad_ws_floats((int)N, (int)H, (int)W, (int)Ci, (int)Co, &ns);
  if (wsf == 0 || N * H * W * std::max(Ci, Co) >= ((int64_t)1 << 31)) return Tensor();
  auto ws = at::empty({wsf}, x.options().dtype(at::kFloat));
  auto dw = at::empty({Co, Ci, 3, 3}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = pdt_conv3x3s2_wgrad(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                     reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                     reinterpret_cast<uint16_t*>(dw.data_ptr()), ws.data_ptr<float>(), (int)N, (int)H,
                                     (int)W, (int)Ci, (int)Co, stream());
  if (rc == -4 || rc == -1 || rc == -2) return Tensor();
  TORCH_CHECK(rc == 0, "pdt_conv3x3s2_wgrad failed: ", rc);
  return dw;
}

// Data-gradient weights: wf [Ci, Co, 3, 3] (channels_last storage [Ci][3][3][Co]) with
// Weight gradient of the stride-1 pad-1 3x3 conv (csrc/kernels/conv3x3_wgrad.hip): dw [Co, Ci, 3, 3]
// channels_last bf16 from channels_last bf16 x [N, Ci, H, W] and dy [N, Co, H, W]. Returns an
// undefined tensor for a shape the kernel does not take (caller falls back).
Tensor conv3x3s1_wgrad(Tensor x, Tensor dy) {
  check_nhwc_bf16(x, "x");
  check_nhwc_bf16(dy, "dy");
  const int64_t N = x.size(0), Ci = x.size(1), H = x.size(2), W = x.size(3), Co = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W, "conv3x3s1_wgrad: dy [N, Co, H, W]");
  int ns = 0;
  const int64_t wsf = pdt_conv3x3_wgrad_ws_floats((int)N, (int)H, (int)W, (int)Ci, (int)Co, &ns);
  if (wsf == 0 || N * H * W * std::max(Ci, Co) >= ((int64_t)1 << 31)) return Tensor();
  auto ws = at::empty({wsf}, x.options().dtype(at::kFloat));
  auto dw = at::empty({Co, Ci, 3, 3}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = pdt_conv3x3s1_wgrad(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                     reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                     reinterpret_cast<uint16_t*>(dw.data_ptr()), ws.data_ptr<float>(), (int)N, (int)H,
                                     (int)W, (int)Ci, (int)Co, stream());
  if (rc == -4) return Tensor();
  TORCH_CHECK(rc == 0, "pdt_conv3x3s1_wgrad failed: ", rc);
  return dw;
}

// wf[ci, co, kh, kw] = w[co, ci, 2 - kh, 2 - kw], so dx = conv3x3s1_fwd(dy, wf).
Tensor conv3x3_flip(Tensor w) {
  check_cuda(w, "w");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.scalar_type() == at::kBFloat16,
              "conv3x3_flip: weight [Co, Ci, 3, 3] bf16");
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t Co = w.size(0), Ci = w.size(1);
  auto wf = at::empty({Ci, Co, 3, 3}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  TORCH_CHECK(pdt_conv3x3_flip_weights(reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                       reinterpret_cast<uint16_t*>(wf.data_ptr()), (int)Co, (int)Ci, stream()) == 0,
              "pdt_conv3x3_flip_weights failed");
  return wf;
}

// ----------------------------------------------------------------------------- 7x7/s2 stem conv (3 -> 64)
// y = conv2d(x, w, stride=2, padding=3) for channels_last bf16 x [N,3,H,W] (W % 32 == 0) and w [64,3,7,7].
Tensor stem_conv_fwd(Tensor x, Tensor w) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.size(1) == 3 && x.size(3) % 32 == 0, "stem_conv: x [N, 3, H, W] with W % 32 == 0");
  TORCH_CHECK(w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7 &&
              w.scalar_type() == at::kBFloat16, "stem_conv: weight [64, 3, 7, 7] bf16");
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3), OH = (H - 1) / 2 + 1, OW = W / 2;
  auto wp = at::empty({pdt_stem_conv_wprep_elems()}, w.options());
  auto y = at::empty({N, 64, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = pdt_stem_conv_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                   reinterpret_cast<uint16_t*>(wp.data_ptr()), reinterpret_cast<uint16_t*>(y.data_ptr()),
                                   (int)N, (int)H, (int)W, stream());
  TORCH_CHECK(rc == 0, "pdt_stem_conv_fwd failed: ", rc);
  return y;
}

// stem_conv_fwd plus the output's BatchNorm statistics -> {y, part} (part: P (2 * 64 + 1) floats, the
// input of bn_relu_maxpool_fwd_parts); {} when it does not apply (W != 224).
std::vector<Tensor> stem_conv_fwd_stats(Tensor x, Tensor w) {
  check_nhwc_bf16(x, "x");
  TORCH_CHECK(x.size(1) == 3 && x.size(3) % 32 == 0, "stem_conv: x [N, 3, H, W] with W % 32 == 0");
  TORCH_CHECK(w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7 &&
              w.scalar_type() == at::kBFloat16, "stem_conv: weight [64, 3, 7, 7] bf16");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3), OH = (H - 1) / 2 + 1, OW = W / 2;
  const int64_t P = pdt_stem_stats_parts((int)N, (int)H, (int)W);
  if (P == 0) return {};
  w = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto wp = at::empty({pdt_stem_conv_wprep_elems()}, w.options());
  auto y = at::empty({N, 64, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto part = at::empty({P * (2 * 64 + 1)}, x.options().dtype(at::kFloat));
  const int rc = pdt_stem_conv_fwd_stats(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                         reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                         reinterpret_cast<uint16_t*>(wp.data_ptr()),
                                         reinterpret_cast<uint16_t*>(y.data_ptr()), part.data_ptr<float>(), (int)N,
                                         (int)H, (int)W, stream());
  TORCH_CHECK(rc == 0, "pdt_stem_conv_fwd_stats failed: ", rc);
  return {y, part};
}

// Weight gradient of stem_conv_fwd: dw [64, 3, 7, 7] (channels_last) from x and dy [N, 64, OH, OW]
// (channels_last); W % 32 == 0 and W <= 224.
Tensor stem_conv_wgrad(Tensor x, Tensor dy) {
  check_nhwc_bf16(x, "x");
  check_nhwc_bf16(dy, "dy");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(x.size(1) == 3 && W % 32 == 0 && W <= 224, "stem_conv_wgrad: x [N, 3, H, W], W % 32 == 0, W <= 224");
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == 64 && dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == W / 2,
              "stem_conv_wgrad: dy [N, 64, OH, OW]");
  auto ws = at::empty({pdt_stem_wgrad_ws_floats()}, x.options().dtype(at::kFloat));
  auto dw = at::empty({64, 3, 7, 7}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = pdt_stem_conv_wgrad(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                     reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                     reinterpret_cast<uint16_t*>(dw.data_ptr()), ws.data_ptr<float>(), (int)N, (int)H,
                                     (int)W, stream());
  TORCH_CHECK(rc == 0, "pdt_stem_conv_wgrad failed: ", rc);
  return dw;
}

// stem_conv_wgrad with the stem BatchNorm's backward apply fused into the gradient load: the conv's
// output gradient is A dz + B (xb - mean) + D (coef [3, 64] = A, B, D from maxpool3s2_bwd_bn_coef;
// xb: the BN input = the stem conv output, dz: the gradient at the BN output, both [N, 64, OH, OW]).
Tensor stem_conv_wgrad_bn(Tensor x, Tensor dz, Tensor xb, Tensor coef, Tensor mean) {
  check_nhwc_bf16(x, "x");
  check_nhwc_bf16(dz, "dz");
  check_nhwc_bf16(xb, "xb");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(x.size(1) == 3 && W % 32 == 0 && W <= 224, "stem_conv_wgrad_bn: x [N, 3, H, W], W % 32 == 0, W <= 224");
  TORCH_CHECK(dz.size(0) == N && dz.size(1) == 64 && dz.size(2) == (H - 1) / 2 + 1 && dz.size(3) == W / 2,
              "stem_conv_wgrad_bn: dz [N, 64, OH, OW]");
  TORCH_CHECK(xb.sizes() == dz.sizes(), "stem_conv_wgrad_bn: xb shape");
  TORCH_CHECK(coef.is_cuda() && coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == 3 * 64,
              "stem_conv_wgrad_bn: coef [3, 64] f32");
  TORCH_CHECK(mean.is_cuda() && mean.scalar_type() == at::kFloat && mean.is_contiguous() && mean.numel() == 64,
              "stem_conv_wgrad_bn: mean [64] f32");
  auto ws = at::empty({pdt_stem_wgrad_ws_floats()}, x.options().dtype(at::kFloat));
  auto dw = at::empty({64, 3, 7, 7}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = pdt_stem_conv_wgrad_bn(
      reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(dz.data_ptr()),
      reinterpret_cast<const uint16_t*>(xb.data_ptr()), coef.data_ptr<float>(), mean.data_ptr<float>(),
      reinterpret_cast<uint16_t*>(dw.data_ptr()), ws.data_ptr<float>(), (int)N, (int)H, (int)W, stream());
  TORCH_CHECK(rc == 0, "pdt_stem_conv_wgrad_bn failed: ", rc);
  return dw;
}

// The same weight gradient from the gradient at the max-pool OUTPUT (dyp [N, 64, PH, PW]) and the pool's
// winner codes: the pool's input gradient dz is formed per tile inside the kernel, never in HBM.
Tensor stem_conv_wgrad_bn_pool(Tensor x, Tensor dyp, Tensor code, Tensor xb, Tensor coef, Tensor mean) {
  check_nhwc_bf16(x, "x");
  check_nhwc_bf16(dyp, "dyp");
  check_nhwc_bf16(xb, "xb");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(x.size(1) == 3 && W % 32 == 0 && W <= 224, "stem_conv_wgrad_bn_pool: x [N, 3, H, W], W % 32 == 0, W <= 224");
  const int64_t OH = (H - 1) / 2 + 1, OW = W / 2;
  TORCH_CHECK(xb.size(0) == N && xb.size(1) == 64 && xb.size(2) == OH && xb.size(3) == OW,
              "stem_conv_wgrad_bn_pool: xb [N, 64, OH, OW]");
  TORCH_CHECK(dyp.size(0) == N && dyp.size(1) == 64 && dyp.size(2) == (OH - 1) / 2 + 1 && dyp.size(3) == (OW - 1) / 2 + 1,
              "stem_conv_wgrad_bn_pool: dyp [N, 64, PH, PW]");
  TORCH_CHECK(code.is_cuda() && code.scalar_type() == at::kByte && code.numel() == dyp.numel() && code.is_contiguous(),
              "stem_conv_wgrad_bn_pool: code uint8, one per dyp element");
  TORCH_CHECK(coef.is_cuda() && coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == 3 * 64,
              "stem_conv_wgrad_bn_pool: coef [3, 64] f32");
  TORCH_CHECK(mean.is_cuda() && mean.scalar_type() == at::kFloat && mean.is_contiguous() && mean.numel() == 64,
              "stem_conv_wgrad_bn_pool: mean [64] f32");
  auto ws = at::empty({pdt_stem_wgrad_ws_floats()}, x.options().dtype(at::kFloat));
  auto dw = at::empty({64, 3, 7, 7}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = pdt_stem_conv_wgrad_bn_pool(
      reinterpret_cast<const uint16_t*>(x.data_ptr()), reinterpret_cast<const uint16_t*>(dyp.data_ptr()),
      code.data_ptr<uint8_t>(), reinterpret_cast<const uint16_t*>(xb.data_ptr()), coef.data_ptr<float>(),
      mean.data_ptr<float>(), reinterpret_cast<uint16_t*>(dw.data_ptr()), ws.data_ptr<float>(), (int)N, (int)H, (int)W,
      stream());
  TORCH_CHECK(rc == 0, "pdt_stem_conv_wgrad_bn_pool failed: ", rc);
  return dw;
}

// ----------------------------------------------------------------------------- cross entropy
std::vector<Tensor> ce_fwd(Tensor logits, Tensor target, double smoothing, int64_t ignore_index) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "ce: logits must be contiguous [N, V]");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous(), "ce: target must be int64");
  const int64_t N = logits.size(0), V = logits.size(1);
  auto fopt = logits.options().dtype(at::kFloat);
  auto loss = at::empty({N}, fopt), lse = at::empty({N}, fopt);
  pdt_ce_fwd(logits.data_ptr(), dcode(logits), target.data_ptr<int64_t>(), N, V, (float)smoothing, ignore_index,
             loss.data_ptr<float>(), lse.data_ptr<float>(), stream());
  return {loss, lse};
}

Tensor ce_bwd(Tensor logits, Tensor target, Tensor lse, c10::optional<Tensor> dloss, double dloss_scale,
              double smoothing, int64_t ignore_index) {
  const int64_t N = logits.size(0), V = logits.size(1);
  auto dl = at::empty_like(logits);
  const float* dp = nullptr;
  Tensor dloss_c;
  if (dloss.has_value() && dloss->defined()) {
    dloss_c = dloss->to(at::kFloat).contiguous();
    if (dloss_c.numel() == 1) dloss_c = dloss_c.expand({N}).contiguous();
    dp = dloss_c.data_ptr<float>();
  }
  pdt_ce_bwd(logits.data_ptr(), dcode(logits), target.data_ptr<int64_t>(), lse.data_ptr<float>(), dp,
             (float)dloss_scale, N, V, (float)smoothing, ignore_index, dl.data_ptr(), stream());
  return dl;
}

// ----------------------------------------------------------------------------- layernorm
// res: optional residual branch; then the sum s = x + res is returned as a 4th output and normalised.
std::vector<Tensor> ln_fwd(Tensor x, Tensor w, Tensor b, double eps, c10::optional<Tensor> res) {
  check_cuda(x, "x");
  TORCH_CHECK(x.is_contiguous(), "ln: x must be contiguous");
  const int64_t D = x.size(-1), N = x.numel() / D;
  TORCH_CHECK(w.scalar_type() == at::kFloat && b.scalar_type() == at::kFloat, "ln: weight/bias must be fp32");
  const bool hr = res.has_value() && res->defined();
  if (hr)
    TORCH_CHECK(res->is_contiguous() && res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type(),
                "ln: residual must match x (contiguous, same shape/dtype)");
  auto y = at::empty_like(x);
  Tensor sum;
  if (hr) sum = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({N}, fopt), rstd = at::empty({N}, fopt);
  int rc = pdt_ln_fwd(x.data_ptr(), hr ? res->data_ptr() : nullptr, dcode(x), w.data_ptr<float>(),
                      b.data_ptr<float>(), y.data_ptr(), hr ? sum.data_ptr() : nullptr, mean.data_ptr<float>(),
                      rstd.data_ptr<float>(), N, (int)D, (float)eps, stream());
  TORCH_CHECK(rc == 0, "pdt_ln_fwd: unsupported D=", D);
  return {y, mean, rstd, sum};
}

// LayerNorm straight to fp8 for an fp8 GEMM (layernorm.hip ln_fwd_fp8_kernel): x bf16 [N, D]
// (+ res: s = x + res stored). Returns {yq [N, D], yq^T [D, N], mean, rstd, s}; state_row is the
// consuming GEMM's input-operand row (amax, scale, ...).
std::vector<Tensor> ln_fwd_fp8(Tensor x, Tensor w, Tensor b, double eps, c10::optional<Tensor> res, Tensor state_row) {
  check_cuda(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.scalar_type() == at::kBFloat16, "ln_fp8: x must be contiguous bf16");
  const int64_t D = x.size(-1), N = x.numel() / D;
  TORCH_CHECK(w.scalar_type() == at::kFloat && b.scalar_type() == at::kFloat, "ln_fp8: weight/bias must be fp32");
  TORCH_CHECK(state_row.scalar_type() == at::kFloat && state_row.numel() >= 3 && state_row.is_contiguous(),
              "ln_fp8: fp32 state row");
  const bool hr = res.has_value() && res->defined();
  if (hr)
    TORCH_CHECK(res->is_contiguous() && res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type(),
                "ln_fp8: residual must match x (contiguous, same shape/dtype)");
  auto o8 = x.options().dtype(at::kFloat8_e4m3fn);
  auto yq = at::empty({N, D}, o8), yqt = at::empty({D, N}, o8);
  Tensor sum;
  if (hr) sum = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto mean = at::empty({N}, fopt), rstd = at::empty({N}, fopt);
  float* st = state_row.data_ptr<float>();
  int rc = pdt_ln_fwd_fp8(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                          hr ? reinterpret_cast<const uint16_t*>(res->data_ptr()) : nullptr, w.data_ptr<float>(),
                          b.data_ptr<float>(), hr ? reinterpret_cast<uint16_t*>(sum.data_ptr()) : nullptr,
                          reinterpret_cast<uint8_t*>(yq.data_ptr()), reinterpret_cast<uint8_t*>(yqt.data_ptr()),
                          mean.data_ptr<float>(), rstd.data_ptr<float>(), N, (int)D, (float)eps, st + 1, st,
                          fp8_striped(state_row), stream());
  TORCH_CHECK(rc == 0, "pdt_ln_fwd_fp8: unsupported N=", N, " D=", D);
  return {yq, yqt, mean, rstd, sum};
}

// dres: optional gradient added into dx (the residual stream's own gradient).
std::vector<Tensor> ln_bwd(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd, c10::optional<Tensor> dres) {
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous(), "ln bwd: contiguous inputs required");
  const int64_t D = x.size(-1), N = x.numel() / D;
  const bool hr = dres.has_value() && dres->defined();
  if (hr)
    TORCH_CHECK(dres->is_contiguous() && dres->sizes() == x.sizes() && dres->scalar_type() == x.scalar_type(),
                "ln bwd: dres must match x (contiguous, same shape/dtype)");
  auto dx = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto dw = at::empty({D}, fopt), db = at::empty({D}, fopt);
  auto ws = at::empty({std::max<int64_t>(pdt_ln_workspace_floats(N, (int)D), 1)}, fopt);
  int rc = pdt_ln_bwd(dy.data_ptr(), x.data_ptr(), hr ? dres->data_ptr() : nullptr, dcode(x), w.data_ptr<float>(),
                      mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(), dw.data_ptr<float>(),
                      db.data_ptr<float>(), N, (int)D, ws.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "pdt_ln_bwd: unsupported D=", D);
  return {dx, dw, db};
}

// ----------------------------------------------------------------------------- bias + gelu
Tensor bias_gelu_fwd(Tensor x, c10::optional<Tensor> bias, bool tanh_form) {
  TORCH_CHECK(x.is_contiguous(), "gelu: x must be contiguous");
  const int64_t D = x.size(-1), N = x.numel() / D;
  auto y = at::empty_like(x);
  const bool hb = bias.has_value() && bias->defined();
  const bool bb = hb && bias->scalar_type() == at::kBFloat16;  // a bf16 model's bias, read as is
  if (hb) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == D && (bb || bias->scalar_type() == at::kFloat),
                "bias_gelu: bias [D] fp32 or bf16");
  }
  int rc = pdt_bias_gelu_fwd(x.data_ptr(), dcode(x), hb ? bias->data_ptr() : nullptr, y.data_ptr(), N, (int)D,
                             tanh_form, stream(), bb ? 1 : 0);
  TORCH_CHECK(rc == 0, "pdt_bias_gelu_fwd failed");
  return y;
}

std::vector<Tensor> bias_gelu_bwd(Tensor dy, Tensor x, c10::optional<Tensor> bias, bool tanh_form) {
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous(), "gelu bwd: contiguous inputs required");
  const int64_t D = x.size(-1), N = x.numel() / D;
  auto dx = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  const bool hb = bias.has_value() && bias->defined();
  const bool bb = hb && bias->scalar_type() == at::kBFloat16;
  Tensor db, ws;
  if (hb) {
    db = at::empty({D}, bb ? x.options().dtype(at::kBFloat16) : fopt);  // the bias's own dtype
    ws = at::empty({pdt_gelu_workspace_floats(N, (int)D)}, fopt);
  }
  int rc = pdt_bias_gelu_bwd(dy.data_ptr(), x.data_ptr(), dcode(x), hb ? bias->data_ptr() : nullptr, dx.data_ptr(),
                             hb ? db.data_ptr() : nullptr, N, (int)D, tanh_form,
                             hb ? ws.data_ptr<float>() : nullptr, stream(), bb ? 1 : 0);
  TORCH_CHECK(rc == 0, "pdt_bias_gelu_bwd failed");
  return {dx, db};
}

// ----------------------------------------------------------------------------- flash attention
// Views are [B, H, T, Dh] bf16 with unit stride on Dh (any b/h/t strides, e.g. slices of a packed qkv).
struct Strides3 {
  int64_t v[3];
};
Strides3 bht_strides(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.dim() == 4 && t.stride(3) == 1, "attn: ", name,
              " must be a bf16 [B,H,T,Dh] view with unit Dh stride");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && t.stride(2) % 8 == 0 && t.stride(1) % 8 == 0,
              "attn: ", name, " rows must be 16-byte aligned");
  return {{t.stride(0), t.stride(1), t.stride(2)}};
}

void attn_fwd_out(Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, bool causal, double scale) {
  auto qs = bht_strides(q, "q"), ks = bht_strides(k, "k"), vs = bht_strides(v, "v"), os = bht_strides(o, "o");
  TORCH_CHECK(q.sizes() == k.sizes() && q.sizes() == v.sizes() && q.sizes() == o.sizes(), "attn: shape mismatch");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == q.size(0) * q.size(1) * q.size(2),
              "attn: lse must be fp32 [B,H,T]");
  const int B = q.size(0), H = q.size(1), T = q.size(2), Dh = q.size(3);
  int rc = pdt_attn_fwd(reinterpret_cast<const uint16_t*>(q.data_ptr()), qs.v, reinterpret_cast<const uint16_t*>(k.data_ptr()),
                        ks.v, reinterpret_cast<const uint16_t*>(v.data_ptr()), vs.v,
                        reinterpret_cast<uint16_t*>(o.data_ptr()), os.v, lse.data_ptr<float>(), B, H, T, Dh, causal,
                        (float)scale, stream());
  TORCH_CHECK(rc == 0, "pdt_attn_fwd: unsupported head dim ", Dh);
}

void attn_bwd_out(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor dq, Tensor dk, Tensor dv,
                  bool causal, double scale) {
  auto dos = bht_strides(dout, "dout"), qs = bht_strides(q, "q"), ks = bht_strides(k, "k"), vs = bht_strides(v, "v"),
       os = bht_strides(o, "o"), gs = bht_strides(dq, "dq"), gk = bht_strides(dk, "dk"), gv = bht_strides(dv, "dv");
  TORCH_CHECK(gs.v[0] == gk.v[0] && gs.v[1] == gk.v[1] && gs.v[2] == gk.v[2] && gs.v[0] == gv.v[0] &&
              gs.v[1] == gv.v[1] && gs.v[2] == gv.v[2], "attn bwd: dq/dk/dv must share strides");
  const int B = q.size(0), H = q.size(1), T = q.size(2), Dh = q.size(3);
  auto delta = at::empty({(int64_t)B * H * T}, q.options().dtype(at::kFloat));
  int rc = pdt_attn_bwd(reinterpret_cast<const uint16_t*>(dout.data_ptr()), dos.v,
                        reinterpret_cast<const uint16_t*>(q.data_ptr()), qs.v, reinterpret_cast<const uint16_t*>(k.data_ptr()),
                        ks.v, reinterpret_cast<const uint16_t*>(v.data_ptr()), vs.v,
                        reinterpret_cast<const uint16_t*>(o.data_ptr()), os.v, lse.data_ptr<float>(),
                        delta.data_ptr<float>(), reinterpret_cast<uint16_t*>(dq.data_ptr()),
                        reinterpret_cast<uint16_t*>(dk.data_ptr()), reinterpret_cast<uint16_t*>(dv.data_ptr()), gs.v, B,
                        H, T, Dh, causal, (float)scale, stream());
  TORCH_CHECK(rc == 0, "pdt_attn_bwd: unsupported head dim ", Dh);
}

// bias gradient of a Linear layer: column sum of dy [*, D] -> [D] in out_dtype (fp32 / bf16)
// xs = x[:, :, ::s, ::s] for a channels_last bf16 [N, C, H, W] tensor (C % 8 == 0), channels_last out.
Tensor subsample_gather(Tensor x, int64_t s) {
  check_nhwc_bf16(x, "x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 8 == 0 && s >= 1, "subsample_gather: C % 8 == 0, s >= 1");
  auto xs = at::empty({N, C, (H - 1) / s + 1, (W - 1) / s + 1}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = pdt_subsample_gather(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                      reinterpret_cast<uint16_t*>(xs.data_ptr()), (int)N, (int)H, (int)W, (int)C,
                                      (int)s, stream());
  TORCH_CHECK(rc == 0, "pdt_subsample_gather failed: ", rc);
  return xs;
}

// full[:, :, ::s, ::s] += t (in place; both channels_last bf16).
void subsample_scatter_add(Tensor t, Tensor full, int64_t s) {
  check_nhwc_bf16(t, "t");
  check_nhwc_bf16(full, "full");
  const int64_t N = full.size(0), C = full.size(1), H = full.size(2), W = full.size(3);
  TORCH_CHECK(t.size(0) == N && t.size(1) == C && t.size(2) == (H - 1) / s + 1 && t.size(3) == (W - 1) / s + 1 &&
              C % 8 == 0, "subsample_scatter_add: shape");
  const int rc = pdt_subsample_scatter_add(reinterpret_cast<const uint16_t*>(t.data_ptr()),
                                           reinterpret_cast<uint16_t*>(full.data_ptr()), (int)N, (int)H, (int)W,
                                           (int)C, (int)s, stream());
  TORCH_CHECK(rc == 0, "pdt_subsample_scatter_add failed: ", rc);
}

// out = x.sum(0) for a contiguous bf16 [S, ...] tensor (S = 2..64, a power of two), fp32 accumulation.
Tensor slice_sum(Tensor x) {
  check_cuda(x, "slice_sum");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() >= 2, "slice_sum: contiguous bf16 [S, ...]");
  const int64_t S = x.size(0), n = x.numel() / S;
  auto out = at::empty(x.sizes().slice(1), x.options());
  const int rc = pdt_slice_sum_bf16(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                    reinterpret_cast<uint16_t*>(out.data_ptr()), (int)S, n, stream());
  TORCH_CHECK(rc == 0, "pdt_slice_sum_bf16 failed: ", rc);
  return out;
}

Tensor colsum(Tensor dy, at::ScalarType out_dtype) {
  check_cuda(dy, "dy");
  TORCH_CHECK(dy.is_contiguous(), "colsum: contiguous input");
  const int64_t D = dy.size(-1), N = D ? dy.numel() / D : 0;
  auto out = at::empty({D}, dy.options().dtype(out_dtype));
  auto ws = at::empty({std::max<int64_t>(pdt_gelu_workspace_floats(N, (int)D), 1)}, dy.options().dtype(at::kFloat));
  int rc = pdt_colsum(dy.data_ptr(), dcode(dy), N, (int)D, out.data_ptr(), dcode(out), ws.data_ptr<float>(),
                      stream());
  TORCH_CHECK(rc == 0, "pdt_colsum failed (D % 8 != 0?)");
  return out;
}

// ---- fp8 (OCP e4m3fn) casts: csrc/kernels/fp8.hip ----
// x: bf16 [M, K] contiguous; state_row: fp32 view [3 + L] = (amax, scale, scale_inv, history...)
// returns {x_fp8 [M, K], x_fp8_t [K, M] (if transpose)}
std::vector<Tensor> fp8_cast_transpose(Tensor x, Tensor state_row, bool transpose) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous(), "fp8_cast: bf16 [M, K]");
  TORCH_CHECK(state_row.scalar_type() == at::kFloat && state_row.numel() >= 3 && state_row.is_contiguous(),
              "fp8_cast: fp32 state row");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(M % 16 == 0 && K % 16 == 0, "fp8_cast: M and K must be multiples of 16");
  auto o8 = x.options().dtype(at::kFloat8_e4m3fn);
  auto out = at::empty({M, K}, o8);
  Tensor out_t;
  if (transpose) out_t = at::empty({K, M}, o8);
  float* st = state_row.data_ptr<float>();
  int rc = pdt_fp8_cast_transpose(reinterpret_cast<const uint16_t*>(x.data_ptr()), M, K, st + 1,
                                  reinterpret_cast<uint8_t*>(out.data_ptr()),
                                  transpose ? reinterpret_cast<uint8_t*>(out_t.data_ptr()) : nullptr, st,
                                  fp8_striped(state_row), stream());
  TORCH_CHECK(rc == 0, "pdt_fp8_cast_transpose failed");
  return {out, out_t};
}

// The MLP activation straight to fp8 (fp8.hip fp8_gelu_cast_kernel). h: bf16 [M, D] (fc1 output
// without bias), bias: fp32 [D] or none. Forward (dg undefined): {fp8(gelu(h + bias)), its
// transpose}. Backward: {fp8(dg * gelu'(h + bias)), its transpose, bias gradient in db_dtype (or
// undefined without bias)}. state_row as fp8_cast_transpose.
std::vector<Tensor> fp8_gelu_cast(Tensor h, c10::optional<Tensor> dg, c10::optional<Tensor> bias, Tensor state_row,
                                  bool tanh_form, at::ScalarType db_dtype) {
  check_cuda(h, "h");
  TORCH_CHECK(h.scalar_type() == at::kBFloat16 && h.dim() == 2 && h.is_contiguous(), "fp8_gelu_cast: bf16 [M, D] h");
  TORCH_CHECK(state_row.scalar_type() == at::kFloat && state_row.numel() >= 3 && state_row.is_contiguous(),
              "fp8_gelu_cast: fp32 state row");
  const int64_t M = h.size(0), D = h.size(1);
  TORCH_CHECK(M % 16 == 0 && D % 64 == 0 && M > 0, "fp8_gelu_cast: M % 16 == 0 and D % 64 == 0");
  const bool bwd = dg.has_value() && dg->defined();
  if (bwd)
    TORCH_CHECK(dg->scalar_type() == at::kBFloat16 && dg->sizes() == h.sizes() && dg->is_contiguous(),
                "fp8_gelu_cast: dg like h");
  const bool hb = bias.has_value() && bias->defined();
  if (hb)
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == D,
                "fp8_gelu_cast: fp32 bias [D]");
  auto o8 = h.options().dtype(at::kFloat8_e4m3fn);
  auto out = at::empty({M, D}, o8), out_t = at::empty({D, M}, o8);
  Tensor part, db;
  if (bwd) part = at::empty({pdt_fp8_gelu_cast_workspace_floats(M, (int)D)}, h.options().dtype(at::kFloat));
  float* st = state_row.data_ptr<float>();
  const int nchunk = pdt_fp8_gelu_cast(reinterpret_cast<const uint16_t*>(h.data_ptr()),
                                       bwd ? reinterpret_cast<const uint16_t*>(dg->data_ptr()) : nullptr,
                                       hb ? bias->data_ptr<float>() : nullptr, M, (int)D, tanh_form, st + 1,
                                       reinterpret_cast<uint8_t*>(out.data_ptr()),
                                       reinterpret_cast<uint8_t*>(out_t.data_ptr()), st,
                                       bwd ? part.data_ptr<float>() : nullptr, fp8_striped(state_row), stream());
  TORCH_CHECK(nchunk > 0, "pdt_fp8_gelu_cast failed: ", nchunk);
  if (bwd && hb) {
    TORCH_CHECK(db_dtype == at::kFloat || db_dtype == at::kBFloat16, "fp8_gelu_cast: db dtype fp32 / bf16");
    db = at::empty({D}, h.options().dtype(db_dtype));
    pdt_colsum_finalize(part.data_ptr<float>(), nchunk, (int)D, db.data_ptr(), db_dtype == at::kFloat ? 0 : 1,
                        stream());
  }
  return {out, out_t, db};
}

// A Linear's output gradient dy (bf16 [M, D], D % 64 == 0): {fp8(dy), its transpose, sum_m dy in
// db_dtype} in one pass (fp8.hip M_CAST_SUM) — the cast and the bias gradient.
std::vector<Tensor> fp8_cast_colsum(Tensor x, Tensor state_row, at::ScalarType db_dtype) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous(), "fp8_cast_colsum: bf16 [M, D]");
  TORCH_CHECK(state_row.scalar_type() == at::kFloat && state_row.numel() >= 3 && state_row.is_contiguous(),
              "fp8_cast_colsum: fp32 state row");
  TORCH_CHECK(db_dtype == at::kFloat || db_dtype == at::kBFloat16, "fp8_cast_colsum: db dtype fp32 / bf16");
  const int64_t M = x.size(0), D = x.size(1);
  TORCH_CHECK(M % 16 == 0 && D % 64 == 0 && M > 0, "fp8_cast_colsum: M % 16 == 0 and D % 64 == 0");
  auto o8 = x.options().dtype(at::kFloat8_e4m3fn);
  auto out = at::empty({M, D}, o8), out_t = at::empty({D, M}, o8);
  auto part = at::empty({pdt_fp8_gelu_cast_workspace_floats(M, (int)D)}, x.options().dtype(at::kFloat));
  auto db = at::empty({D}, x.options().dtype(db_dtype));
  float* st = state_row.data_ptr<float>();
  const int nchunk = pdt_fp8_cast_colsum(reinterpret_cast<const uint16_t*>(x.data_ptr()), M, (int)D, st + 1,
                                         reinterpret_cast<uint8_t*>(out.data_ptr()),
                                         reinterpret_cast<uint8_t*>(out_t.data_ptr()), st, part.data_ptr<float>(),
                                         fp8_striped(state_row), stream());
  TORCH_CHECK(nchunk > 0, "pdt_fp8_cast_colsum failed: ", nchunk);
  pdt_colsum_finalize(part.data_ptr<float>(), nchunk, (int)D, db.data_ptr(), db_dtype == at::kFloat ? 0 : 1, stream());
  return {out, out_t, db};
}

// Every tensor of xs (bf16 [M_i, K_i] contiguous) cast with its state row in one launch (<= 64 per
// launch): returns [q_0, qt_0, q_1, qt_1, ...].
std::vector<Tensor> fp8_cast_multi(std::vector<Tensor> xs, std::vector<Tensor> rows) {
  TORCH_CHECK(xs.size() == rows.size(), "fp8_cast_multi: one state row per tensor");
  std::vector<Tensor> res;
  res.reserve(2 * xs.size());
  for (size_t base = 0; base < xs.size(); base += 64) {
    const int n = (int)std::min<size_t>(64, xs.size() - base);
    std::vector<const uint16_t*> px(n);
    std::vector<int> pm(n), pk(n), pst(n);
    std::vector<float*> ps(n);
    std::vector<uint8_t*> po(n), pt(n);
    for (int i = 0; i < n; ++i) {
      const Tensor& x = xs[base + i];
      const Tensor& r = rows[base + i];
      check_cuda(x, "x");
      TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous(), "fp8_cast_multi: bf16 [M, K]");
      TORCH_CHECK(r.scalar_type() == at::kFloat && r.numel() >= 3 && r.is_contiguous(), "fp8_cast_multi: state row");
      const int64_t M = x.size(0), K = x.size(1);
      TORCH_CHECK(M % 16 == 0 && K % 16 == 0 && M > 0 && M * K < ((int64_t)1 << 31), "fp8_cast_multi: shape");
      auto o8 = x.options().dtype(at::kFloat8_e4m3fn);
      res.push_back(at::empty({M, K}, o8));
      res.push_back(at::empty({K, M}, o8));
      px[i] = reinterpret_cast<const uint16_t*>(x.data_ptr());
      pm[i] = (int)M;
      pk[i] = (int)K;
      ps[i] = r.data_ptr<float>();
      pst[i] = fp8_striped(r);
      po[i] = reinterpret_cast<uint8_t*>(res[res.size() - 2].data_ptr());
      pt[i] = reinterpret_cast<uint8_t*>(res.back().data_ptr());
    }
    const int rc = pdt_fp8_cast_multi(n, px.data(), pm.data(), pk.data(), ps.data(), pst.data(), po.data(), pt.data(),
                                      stream());
    TORCH_CHECK(rc == 0, "pdt_fp8_cast_multi failed: ", rc);
  }
  return res;
}

void fp8_update_scales(Tensor state, int64_t history, double margin) {
  check_cuda(state, "state");
  const bool striped = state.dim() == 2 && state.size(1) == kFp8StripedRow - 1 + history;
  TORCH_CHECK(state.scalar_type() == at::kFloat && state.is_contiguous() && state.dim() == 2 &&
                  (state.size(1) == 3 + history || striped),
              "fp8_update_scales: state [n, 3 + L] or striped [n, 260 + L] fp32");
  pdt_fp8_update_scales(state.data_ptr<float>(), (int)state.size(0), (int)history, (float)std::pow(2.0, margin),
                        striped ? 1 : 0, stream());
}

// ---- intra-node P2P all-reduce (csrc/kernels/p2p.hip) ----
#define PDT_HIP_CHECK(expr)                                                            \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    TORCH_CHECK(e_ == hipSuccess, "pdt p2p: ", #expr, " failed: ", hipGetErrorString(e_)); \
  } while (0)

struct DevGuard {  // select `dev` for the scope, restore the caller's device after
  int prev = 0;
  explicit DevGuard(int dev) {
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(dev);
  }
  ~DevGuard() { (void)hipSetDevice(prev); }
};

class P2PComm {
 public:
  P2PComm(int rank, int world, int64_t capacity_bytes, int max_blocks, int device)
      : rank_(rank), world_(world), cap_(capacity_bytes), max_blocks_(max_blocks), device_(device) {
    TORCH_CHECK(world >= 1 && world <= 8 && rank >= 0 && rank < world, "p2p: 1 <= world <= 8");
    TORCH_CHECK(capacity_bytes % 16 == 0, "p2p: capacity must be a multiple of 16 bytes");
    DevGuard guard(device_);
    flags_bytes_ = pdt_p2p_flags_bytes();
    // uncached: peers poll/read these over xGMI; no stale L2 lines on either side
    PDT_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), flags_bytes_, hipDeviceMallocUncached));
    PDT_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&data_), pdt_p2p_data_bytes(cap_),
                                        hipDeviceMallocUncached));
    PDT_HIP_CHECK(hipMemset(flags_, 0, flags_bytes_));
    PDT_HIP_CHECK(hipDeviceSynchronize());
    data_ptrs_.assign(world_, nullptr);
    flag_ptrs_.assign(world_, nullptr);
    data_ptrs_[rank_] = data_;
    flag_ptrs_[rank_] = flags_;
  }
  ~P2PComm() {
    for (int r = 0; r < world_; ++r)
      if (r != rank_) {
        if (data_ptrs_[r]) (void)hipIpcCloseMemHandle(data_ptrs_[r]);
        if (flag_ptrs_[r]) (void)hipIpcCloseMemHandle(flag_ptrs_[r]);
      }
    (void)hipFree(flags_);
    (void)hipFree(data_);
  }
  // 2 x hipIpcMemHandle_t (data, flags) as bytes, to be exchanged through the c10d store
  py::bytes handles() const {
    hipIpcMemHandle_t h[2];
    PDT_HIP_CHECK(hipIpcGetMemHandle(&h[0], data_));
    PDT_HIP_CHECK(hipIpcGetMemHandle(&h[1], flags_));
    return py::bytes(reinterpret_cast<const char*>(h), sizeof(h));
  }
  void open(const std::vector<py::bytes>& all) {
    TORCH_CHECK((int)all.size() == world_, "p2p: need one handle blob per rank");
    DevGuard guard(device_);
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      std::string b = all[r];
      TORCH_CHECK(b.size() == 2 * sizeof(hipIpcMemHandle_t), "p2p: bad handle blob");
      hipIpcMemHandle_t h[2];
      std::memcpy(h, b.data(), sizeof(h));
      void* d = nullptr;
      void* f = nullptr;
      PDT_HIP_CHECK(hipIpcOpenMemHandle(&d, h[0], hipIpcMemLazyEnablePeerAccess));
      PDT_HIP_CHECK(hipIpcOpenMemHandle(&f, h[1], hipIpcMemLazyEnablePeerAccess));
      data_ptrs_[r] = static_cast<char*>(d);
      flag_ptrs_[r] = static_cast<uint32_t*>(f);
    }
    opened_ = true;
  }
  // out = post_scale * sum over ranks of `in` (out may alias in); enqueued on the current stream.
  // st: int32 [3] device state owned by the caller, zero-initialised ([0] epoch, [1] finished-block
  // counter, [2] sticky error flag) — advanced by the kernel itself (hipGraph-capture safe).
  // algo 0 = one-shot, 1 = two-shot (reduce-scatter + all-gather).
  void allreduce(Tensor in, Tensor out, double post_scale, Tensor st, int64_t algo, double timeout_s) {
    TORCH_CHECK(opened_ || world_ == 1, "p2p: open() the peer handles first");
    check_cuda(in, "in");
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel() &&
                    in.scalar_type() == out.scalar_type(), "p2p: contiguous in/out of equal size and dtype");
    TORCH_CHECK(in.numel() % 8 == 0, "p2p: numel must be a multiple of 8");
    TORCH_CHECK(in.numel() * in.element_size() <= cap_, "p2p: tensor larger than the staging capacity");
    check_cuda(st, "st");
    TORCH_CHECK(st.scalar_type() == at::kInt && st.numel() >= 3 && st.is_contiguous(), "p2p: st int32 [3]");
    TORCH_CHECK(algo == 0 || algo == 1, "p2p: algo 0 (one-shot) or 1 (two-shot)");
    int rc = pdt_p2p_allreduce(in.data_ptr(), out.data_ptr(), in.numel(), dcode(in), data_ptrs_.data(),
                               flag_ptrs_.data(), rank_, world_, cap_, (float)post_scale,
                               reinterpret_cast<uint32_t*>(st.data_ptr<int>()), (int)algo, max_blocks_, timeout_s,
                               stream());
    TORCH_CHECK(rc == 0, "pdt_p2p_allreduce failed (", rc, ")");
  }
  int64_t capacity() const { return cap_; }

 private:
  int rank_, world_;
  int64_t cap_;
  int max_blocks_, device_;
  int64_t flags_bytes_ = 0;
  char* data_ = nullptr;
  uint32_t* flags_ = nullptr;
  bool opened_ = false;
  std::vector<char*> data_ptrs_;
  std::vector<uint32_t*> flag_ptrs_;
};

// ---- GPT-2 token + position embedding (csrc/kernels/embedding.hip) ----
// out [B, T, D] = wte[idx] + wpe[arange(T)] (bf16). idx int64 [B, T]; values must be < V (checked on
// the host only in debug paths: an out-of-range id is a caller bug, as for nn.Embedding).
// Per-device error word of the embedding kernels (an out-of-range token id sets it; never cleared
// by the kernels). Allocated at the first call (before any graph capture of the model).
Tensor embedding_err(const Tensor& like) {
  static std::map<int, Tensor> bufs;
  const int dev = like.get_device();
  auto it = bufs.find(dev);
  if (it == bufs.end()) it = bufs.emplace(dev, at::zeros({1}, like.options().dtype(at::kInt))).first;
  return it->second;
}

Tensor embedding_fwd(Tensor idx, Tensor wte, Tensor wpe) {
  check_cuda(idx, "idx");
  check_cuda(wte, "wte");
  check_cuda(wpe, "wpe");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 2 && idx.is_contiguous(), "embedding: idx int64 [B, T]");
  TORCH_CHECK(wte.scalar_type() == at::kBFloat16 && wpe.scalar_type() == at::kBFloat16 && wte.is_contiguous() &&
                  wpe.is_contiguous() && wte.dim() == 2 && wpe.dim() == 2 && wte.size(1) == wpe.size(1),
              "embedding: wte [V, D], wpe [P, D] contiguous bf16");
  const int64_t B = idx.size(0), T = idx.size(1), D = wte.size(1);
  TORCH_CHECK(T <= wpe.size(0) && D % 8 == 0, "embedding: T <= P, D % 8 == 0");
  auto out = at::empty({B, T, D}, wte.options());
  TORCH_CHECK(pdt_embedding_fwd(idx.data_ptr<int64_t>(), reinterpret_cast<const uint16_t*>(wte.data_ptr()),
                                reinterpret_cast<const uint16_t*>(wpe.data_ptr()),
                                reinterpret_cast<uint16_t*>(out.data_ptr()), B * T, (int)T, (int)D, (int)wte.size(0),
                                embedding_err(idx).data_ptr<int>(), stream()) == 0,
              "pdt_embedding_fwd failed");
  return out;
}

// (dwte [V, D], dwpe [P, D]) from dout [B, T, D]: deterministic (counting sort + ordered row sums).
std::vector<Tensor> embedding_bwd(Tensor idx, Tensor dout, int64_t V, int64_t P) {
  check_cuda(idx, "idx");
  check_cuda(dout, "dout");
  dout = dout.contiguous();
  TORCH_CHECK(dout.scalar_type() == at::kBFloat16 && dout.dim() == 3 && dout.size(0) == idx.size(0) &&
                  dout.size(1) == idx.size(1), "embedding_bwd: dout [B, T, D] bf16");
  const int64_t B = idx.size(0), T = idx.size(1), D = dout.size(2), n = B * T;
  auto ws = at::zeros({pdt_embedding_bwd_ws_ints(n, (int)V)}, idx.options().dtype(at::kInt));
  auto dwte = at::empty({V, D}, dout.options());
  auto dwpe = T == P ? at::empty({P, D}, dout.options()) : at::zeros({P, D}, dout.options());
  TORCH_CHECK(pdt_embedding_bwd(idx.data_ptr<int64_t>(), reinterpret_cast<const uint16_t*>(dout.data_ptr()),
                                reinterpret_cast<uint16_t*>(dwte.data_ptr()), reinterpret_cast<uint16_t*>(dwpe.data_ptr()),
                                ws.data_ptr<int>(), n, (int)B, (int)T, (int)V, (int)D,
                                embedding_err(idx).data_ptr<int>(), stream()) == 0,
              "pdt_embedding_bwd failed");
  return {dwte, dwpe};
}

// ---- Linear GEMM with fused epilogues (csrc/kernels/gemm.hip) ----
// a [M, K], b [N, K] contiguous bf16 -> {C [M, N]} (epi 0: a·bᵀ, 1: a·bᵀ + bias) or {C, G} (epi 2:
// C = a·bᵀ, G = gelu(C + bias)). bias [N] fp32 or bf16. N % 256 == 0, K % 64 == 0 (gemm_nt_ok).
std::vector<Tensor> gemm_nt(Tensor a, Tensor b, c10::optional<Tensor> bias, int64_t epi, bool tanh_form) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && a.dim() == 2 && b.dim() == 2 &&
                  a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
              "gemm_nt: a [M, K], b [N, K] contiguous bf16");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  const void* bp = nullptr;
  int bf32 = 0;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N &&
                    (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16),
                "gemm_nt: bias [N] fp32 or bf16");
    bp = bias->data_ptr();
    bf32 = bias->scalar_type() == at::kFloat;
  }
  auto c = at::empty({M, N}, a.options());
  Tensor g = epi == 2 ? at::empty({M, N}, a.options()) : Tensor();
  const int rc = pdt_gemm_nt(reinterpret_cast<const uint16_t*>(a.data_ptr()), reinterpret_cast<const uint16_t*>(b.data_ptr()),
                             reinterpret_cast<uint16_t*>(c.data_ptr()),
                             epi == 2 ? reinterpret_cast<uint16_t*>(g.data_ptr()) : nullptr, bp, bf32, (int)epi,
                             tanh_form ? 1 : 0, (int)M, (int)N, (int)K, stream());
  TORCH_CHECK(rc == 0, "pdt_gemm_nt failed (", rc, ") for M=", M, " N=", N, " K=", K);
  if (epi == 2) return {c, g};
  return {c};
}

// fp8 e4m3 operands (csrc/kernels/gemm.hip F8): C [M, N] bf16 = (a sa)(b sb)^T (+ bias) from a [M, K], b [N, K]
// contiguous float8_e4m3fn and one-element fp32 dequantisation scales (torch._scaled_mm's scale_a / scale_b).
// N % 128 == 0, K % 128 == 0 (gemm_nt_fp8_ok).
Tensor gemm_nt_fp8(Tensor a, Tensor b, Tensor sa, Tensor sb, c10::optional<Tensor> bias) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  TORCH_CHECK(a.scalar_type() == at::kFloat8_e4m3fn && b.scalar_type() == at::kFloat8_e4m3fn && a.dim() == 2 &&
                  b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
              "gemm_nt_fp8: a [M, K], b [N, K] contiguous float8_e4m3fn");
  TORCH_CHECK(sa.scalar_type() == at::kFloat && sb.scalar_type() == at::kFloat && sa.numel() == 1 && sb.numel() == 1 &&
                  sa.is_cuda() && sb.is_cuda(), "gemm_nt_fp8: one-element fp32 device scales");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  const void* bp = nullptr;
  int bf32 = 0;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N &&
                    (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16),
                "gemm_nt_fp8: bias [N] fp32 or bf16");
    bp = bias->data_ptr();
    bf32 = bias->scalar_type() == at::kFloat;
  }
  auto c = at::empty({M, N}, a.options().dtype(at::kBFloat16));
  // few output tiles and no bias (the weight gradients): split K, fp32 partials + one reduce pass
  const int ks = bp ? 1 : pdt_gemm_nt_fp8_ksplit((int)M, (int)N, (int)K);
  Tensor ws;
  if (ks > 1) ws = at::empty({(int64_t)ks * M * N}, a.options().dtype(at::kFloat));
  const int rc = pdt_gemm_nt_fp8(reinterpret_cast<const uint8_t*>(a.data_ptr()), reinterpret_cast<const uint8_t*>(b.data_ptr()),
                                 reinterpret_cast<uint16_t*>(c.data_ptr()), sa.data_ptr<float>(), sb.data_ptr<float>(), bp,
                                 bf32, bp ? 1 : 0, (int)M, (int)N, (int)K, ks > 1 ? ws.data_ptr<float>() : nullptr, ks,
                                 stream());
  TORCH_CHECK(rc == 0, "pdt_gemm_nt_fp8 failed (", rc, ") for M=", M, " N=", N, " K=", K);
  return c;
}

// ---- LeNet (reference model) ops: csrc/kernels/lenet.hip ----
constexpr int kStemIpb = 4;  // images per workgroup in the conv1 weight-gradient reduction

std::vector<Tensor> lenet_stem_fwd(Tensor x, Tensor w, Tensor b, double slope) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4 && x.size(1) == 1 &&
                  x.size(2) == 28 && x.size(3) == 28, "lenet_stem: x must be contiguous fp32 [N,1,28,28]");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == 150 && b.numel() == 6 &&
                  b.is_contiguous(), "lenet_stem: conv1 weight [6,1,5,5] / bias [6] fp32");
  const int64_t N = x.size(0);
  auto y = at::empty({N, 6, 14, 14}, x.options());
  auto code = at::empty({N, 6, 14, 14}, x.options().dtype(at::kByte));
  pdt_lenet_stem_fwd(x.data_ptr<float>(), w.data_ptr<float>(), b.data_ptr<float>(), N, (float)slope,
                     y.data_ptr<float>(), code.data_ptr<uint8_t>(), stream());
  return {y, code};
}

std::vector<Tensor> lenet_stem_bwd(Tensor dy, Tensor code, Tensor x, double slope) {
  const int64_t N = x.size(0);
  dy = dy.contiguous();
  TORCH_CHECK(dy.scalar_type() == at::kFloat && dy.numel() == N * 1176 && code.numel() == N * 1176 &&
                  x.numel() == N * 784, "lenet_stem_bwd: shape mismatch");
  auto slab = at::empty({std::max<int64_t>(pdt_lenet_stem_slab_floats(N, kStemIpb), 1)}, x.options());
  auto dw = at::empty({6, 1, 5, 5}, x.options());
  auto db = at::empty({6}, x.options());
  pdt_lenet_stem_bwd(dy.data_ptr<float>(), code.data_ptr<uint8_t>(), x.data_ptr<float>(), N, kStemIpb,
                     (float)slope, slab.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(), stream());
  return {dw, db};
}

std::vector<Tensor> leaky_pool_fwd(Tensor x, double slope) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4, "leaky_pool: contiguous fp32 NCHW");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  auto y = at::empty({N, C, H / 2, W / 2}, x.options());
  auto code = at::empty({N, C, H / 2, W / 2}, x.options().dtype(at::kByte));
  pdt_leaky_pool_fwd(x.data_ptr<float>(), N * C, (int)H, (int)W, (float)slope, y.data_ptr<float>(),
                     code.data_ptr<uint8_t>(), stream());
  return {y, code};
}

Tensor leaky_pool_bwd(Tensor dy, Tensor code, int64_t H, int64_t W, double slope) {
  dy = dy.contiguous();
  const int64_t N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(dy.scalar_type() == at::kFloat && dy.size(2) == H / 2 && dy.size(3) == W / 2 &&
                  code.numel() == dy.numel(), "leaky_pool_bwd: shape mismatch");
  auto dx = at::empty({N, C, H, W}, dy.options());
  pdt_leaky_pool_bwd(dy.data_ptr<float>(), code.data_ptr<uint8_t>(), N * C, (int)H, (int)W, (float)slope,
                     dx.data_ptr<float>(), stream());
  return dx;
}

// returns {loss[N] (if want_loss), dlogits (if want_grad)}; acc (fp64 [3]) accumulates eval metrics
// mean_scale > 0 (with want_loss): also {.., mean_scale * sum(loss)} as a 0-d fp32 tensor (fixed-order
// one-workgroup sum; the training loss without a torch reduction per step).
std::vector<Tensor> softmax_nll_small(Tensor logits, Tensor target, int64_t mode, double smoothing, bool want_loss,
                                      bool want_grad, double dscale, c10::optional<Tensor> acc,
                                      double mean_scale) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "softmax_nll_small: contiguous [N, V] logits");
  TORCH_CHECK(logits.size(1) <= 1024, "softmax_nll_small: V <= 1024");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous(), "softmax_nll_small: int64 target");
  const int64_t N = logits.size(0);
  Tensor loss, dl;
  if (want_loss) loss = at::empty({N}, logits.options().dtype(at::kFloat));
  if (want_grad) dl = at::empty_like(logits);
  double* ap = nullptr;
  if (acc.has_value() && acc->defined()) {
    TORCH_CHECK(acc->scalar_type() == at::kDouble && acc->numel() >= 3, "softmax_nll_small: acc fp64 [3]");
    ap = acc->data_ptr<double>();
  }
  int rc = pdt_softmax_nll_small(logits.data_ptr(), dcode(logits), target.data_ptr<int64_t>(), N,
                                 (int)logits.size(1), (int)mode, (float)smoothing,
                                 want_loss ? loss.data_ptr<float>() : nullptr, want_grad ? dl.data_ptr() : nullptr,
                                 (float)dscale, ap, stream());
  TORCH_CHECK(rc == 0, "pdt_softmax_nll_small failed");
  if (mean_scale > 0.0 && want_loss) {
    auto mean = at::empty({}, logits.options().dtype(at::kFloat));
    pdt_mean_small(loss.data_ptr<float>(), N, (float)mean_scale, mean.data_ptr<float>(), stream());
    return {loss, dl, mean};
  }
  return {loss, dl};
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels for pytorch_distributed_training_example_amd";
  m.def("sgd", &sgd);
  m.def("adam", &adam);
  m.def("adadelta", &adadelta);
  m.def("amp_unscale", &amp_unscale);
  m.def("amp_update", &amp_update);
  m.def("mt_scale", &mt_scale);
  m.def("mt_copy", &mt_copy);
  m.def("l2norm_sq", &l2norm_sq);
  m.def("clip_coef", &clip_coef);
  m.def("bn_tune", [](int variant, int target_blocks, int u_fwd, int u_bwd) {
    pdt_bn_tune(variant, target_blocks, u_fwd, u_bwd);
  }, py::arg("variant") = 0, py::arg("target_blocks") = 0, py::arg("u_fwd") = 0, py::arg("u_bwd") = 0);
  m.def("bn_fwd_train", &bn_fwd_train, py::arg("x"), py::arg("res"), py::arg("weight"), py::arg("bias"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"), py::arg("relu"),
        py::arg("res_ab") = py::none(), py::arg("apply") = true);
  m.def("bn_fwd_eval", &bn_fwd_eval);
  m.def("bn_relu_maxpool_fwd", &bn_relu_maxpool_fwd);
  m.def("bn_relu_maxpool_fwd_parts", &bn_relu_maxpool_fwd_parts);
  m.def("maxpool3s2_bwd", &maxpool3s2_bwd);
  m.def("conv1x1_gemm", &conv1x1_gemm, py::arg("a"), py::arg("b"), py::arg("out"), py::arg("acc"), py::arg("stats"),
        py::arg("c_in") = py::none(), py::arg("c_mask") = py::none(), py::arg("bn_x") = py::none(),
        py::arg("bn_mask") = py::none(), py::arg("bn_mean") = py::none(), py::arg("c_stride") = 0,
        py::arg("c_H") = 0, py::arg("c_W") = 0, py::arg("a_coef") = py::none(), py::arg("bn_sum_only") = false,
        py::arg("no_store") = false);
  m.def("conv1x1_probe", [](int probe) { pdt_conv1x1_probe(probe); });
  m.def("conv1x1_persist", [](int mode) { return pdt_conv1x1_persist(mode); },
        "1x1 GEMM persistence mode (0 off, 1 measured kinds, 2 all, -1 env default); returns the previous mode");
  m.def("conv3x3_opt", [](int v) { return pdt_conv3x3_opt(v); },
        "3x3 conv variant bits (csrc/kernels/conv3x3.hip conv3x3_opt; -1 env default); returns the previous value");
  m.def("weight_prep", &weight_prep);
  m.def("bn_tiles_fused", [](int on) { pdt_bn_tiles_fused(on); });
  m.def("maxpool_bwd_v2", [](int on) { pdt_maxpool_bwd_v2(on); });
  m.def("pool_fwd_contig", [](int on) { pdt_pool_fwd_contig(on); });
  m.def("bn_apply_wgs", [](int n) { pdt_bn_apply_wgs(n); });
  m.def("bn_row_wgs", [](int n) { pdt_bn_row_wgs(n); });
  m.def("gap_bwd", &gap_bwd, py::arg("g"), py::arg("H"), py::arg("W"), py::arg("bn_x") = py::none(),
        py::arg("bn_mask") = py::none(), py::arg("bn_mean") = py::none(), py::arg("bn_sum_only") = false);
  m.def("conv1x1_gemm_apply", &conv1x1_gemm_apply, py::arg("a"), py::arg("b"), py::arg("res"), py::arg("ab"),
        py::arg("rab") = py::none(), py::arg("a_coef") = py::none());
  m.def("bn_bwd_train_tiles", &bn_bwd_train_tiles);
  m.def("maxpool3s2_bwd_bn", &maxpool3s2_bwd_bn);
  m.def("maxpool3s2_bwd_bn_coef", &maxpool3s2_bwd_bn_coef, py::arg("dy"), py::arg("code"), py::arg("x"),
        py::arg("weight"), py::arg("mean"), py::arg("invstd"), py::arg("need_dgamma"), py::arg("write_dz") = true);
  m.def("slice_sum", &slice_sum);
  m.def("subsample_gather", &subsample_gather);
  m.def("subsample_scatter_add", &subsample_scatter_add);
  m.def("bn_fwd_train_tiles", &bn_fwd_train_tiles, py::arg("x"), py::arg("part"), py::arg("res"), py::arg("weight"),
        py::arg("bias"), py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"), py::arg("eps"),
        py::arg("relu"), py::arg("res_ab") = py::none(), py::arg("apply") = true, py::arg("sub") = 0);
  m.def("conv3x3s1_fwd", &conv3x3s1_fwd);
  m.def("conv3x3s1_fwd_stats", &conv3x3s1_fwd_stats);
  m.def("conv3x3s1_fwd_bnbwd", &conv3x3s1_fwd_bnbwd);
  m.def("conv3x3_flip", &conv3x3_flip);
  m.def("conv3x3s2_fwd", &conv3x3s2_fwd);
  m.def("conv3x3s2_wgrad", &conv3x3s2_wgrad);
  m.def("conv3x3s2_dgrad", &conv3x3s2_dgrad, py::arg("dy"), py::arg("wf"), py::arg("H"), py::arg("W"),
        py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(), py::arg("bn_mean") = py::none());
  m.def("stem_conv_fwd", &stem_conv_fwd);
  m.def("stem_conv_fwd_stats", &stem_conv_fwd_stats);
  m.def("stem_conv_wgrad", &stem_conv_wgrad);
  m.def("stem_conv_wgrad_bn", &stem_conv_wgrad_bn);
  m.def("stem_conv_wgrad_bn_pool", &stem_conv_wgrad_bn_pool);
  m.def("conv3x3s1_wgrad", &conv3x3s1_wgrad);
  m.def("conv1x1_wgrad", &conv1x1_wgrad);
  m.def("conv1x1_wgrad_seg", &conv1x1_wgrad_seg);
  m.def("conv1x1_gemm_seg", &conv1x1_gemm_seg, py::arg("a1"), py::arg("a2"), py::arg("rep2"), py::arg("b"),
        py::arg("out"), py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(), py::arg("bn_mean") = py::none());
  m.def("bn_alg_assemble", &bn_alg_assemble, py::arg("w"), py::arg("coef"), py::arg("mean"), py::arg("G"), py::arg("wg"),
        py::arg("BWG"), py::arg("rep") = 2);
  m.def("bn_alg_fix_s2", &bn_alg_fix_s2);
  m.def("bn_alg_ds_part", &bn_alg_ds_part);
  m.def("bn_alg_small_gemm", &bn_alg_small_gemm, py::arg("w"), py::arg("coef"), py::arg("wg"), py::arg("wt") = py::none());
  m.def("conv1x1_wgrad_tune", [](int target_wgs, int variant, int interleave) { pdt_conv1x1_wgrad_tune(target_wgs, variant, interleave); },
        py::arg("target_wgs"), py::arg("variant") = -2, py::arg("interleave") = -2);
  m.def("embedding_fwd", &embedding_fwd);
  m.def("gemm_nt", &gemm_nt);
  m.def("gemm_nt_fp8", &gemm_nt_fp8, py::arg("a"), py::arg("b"), py::arg("sa"), py::arg("sb"), py::arg("bias") = py::none());
  m.def("embedding_bwd", &embedding_bwd);
  m.def("embedding_err", &embedding_err);
  m.def("conv3x3_wgrad_tune", [](int target_wgs, int co_tile) { pdt_conv3x3_wgrad_tune(target_wgs, co_tile); });
  m.def("bn_bwd_train", &bn_bwd_train);
  m.def("bn_bwd_coef", &bn_bwd_coef);
  m.def("conv1x1_bwd_fused", &conv1x1_bwd_fused, py::arg("dy"), py::arg("z"), py::arg("mz"), py::arg("mean"),
        py::arg("coef"), py::arg("w"), py::arg("xa"), py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(),
        py::arg("bn_mean") = py::none(), py::arg("xcoef") = py::none(), py::arg("wt") = py::none());
  m.def("conv1x1_bwd_fused_tune", [](int grid) { pdt_conv1x1_bwd_fused_tune(grid); });
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
  m.def("ln_fwd", &ln_fwd, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("eps"), py::arg("res") = py::none());
  m.def("ln_fwd_fp8", &ln_fwd_fp8, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("eps"), py::arg("res"),
        py::arg("state_row"));
  m.def("ln_bwd", &ln_bwd, py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("mean"), py::arg("rstd"),
        py::arg("dres") = py::none());
  m.def("bias_gelu_fwd", &bias_gelu_fwd);
  m.def("bias_gelu_bwd", &bias_gelu_bwd);
  m.def("attn_fwd_out", &attn_fwd_out);
  m.def("attn_bwd_out", &attn_bwd_out);
  m.def("colsum", &colsum);
  py::class_<P2PComm>(m, "P2PComm")
      .def(py::init<int, int, int64_t, int, int>(), py::arg("rank"), py::arg("world"), py::arg("capacity_bytes"),
           py::arg("max_blocks"), py::arg("device"))
      .def("handles", &P2PComm::handles)
      .def("open", &P2PComm::open)
      .def("allreduce", &P2PComm::allreduce)
      .def("capacity", &P2PComm::capacity);
  m.def("fp8_cast_transpose", &fp8_cast_transpose);
  m.def("fp8_update_scales", &fp8_update_scales);
  m.def("fp8_gelu_cast", &fp8_gelu_cast, py::arg("h"), py::arg("dg") = py::none(), py::arg("bias") = py::none(),
        py::arg("state_row"), py::arg("tanh_form") = false, py::arg("db_dtype") = at::kFloat);
  m.def("fp8_cast_multi", &fp8_cast_multi);
  m.def("fp8_cast_colsum", &fp8_cast_colsum);
  m.def("lenet_stem_fwd", &lenet_stem_fwd);
  m.def("lenet_stem_bwd", &lenet_stem_bwd);
  m.def("leaky_pool_fwd", &leaky_pool_fwd);
  m.def("leaky_pool_bwd", &leaky_pool_bwd);
  m.def("lenet_tail_fwd", &lenet_tail_fwd);
  m.def("lenet_tail_bwd", &lenet_tail_bwd);
  m.def("softmax_nll_small", &softmax_nll_small, py::arg("logits"), py::arg("target"), py::arg("mode"),
        py::arg("smoothing"), py::arg("want_loss"), py::arg("want_grad"), py::arg("dscale"), py::arg("acc"),
        py::arg("mean_scale") = 0.0);
}
