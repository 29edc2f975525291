/*
 * nfx.h — C-ABI of libnfx.so, the MI355X (gfx950) flow-transform hot path.
 *
 * The reference (itxtx/normalizing-flows-study) has no native boundary: its hot path is the
 * Python `Flow` contract `forward(z) -> (x, log_det)` / `inverse(x) -> (z, log_det)`
 * (src/flows/flow/flow.py:12-38). Each entry point below replaces the ATen op chain of one
 * reference layer method; the Python mirror in normalizing-flows-study_amd/nfs_amd binds them
 * with ctypes (INTEGRATION.md shows the same stub for the reference tree).
 *
 * Conventions (all entry points):
 *   - Every tensor pointer is a DEVICE pointer owned by the caller (PyTorch allocator).
 *     The library allocates nothing persistent and frees nothing.
 *   - Tensors are fp32, row-major and contiguous: x/z `[B, d]`, log_det `[B]`.
 *   - `stream` is a hipStream_t (0 = null stream). Every call is stream-ordered and
 *     asynchronous; no call synchronises the device, so calls can be captured in a hipGraph.
 *   - Return 0 on success; < 0 on error, with a message in nfx_last_error() (thread-local).
 *     NFX_EINVAL invalid argument, NFX_EUNSUPPORTED shape outside the compiled kernel
 *     family, NFX_ELAUNCH a HIP launch error.
 *   - `accumulate` = 0 stores the layer's log|det J| into log_det; 1 adds it in place
 *     (log_det[i] += ld_i), reproducing the sequential float32 accumulation of
 *     NormalizingFlowModel.forward/inverse (src/models/normalizing_flow_model.py:30-65).
 *   - `direction` = NFX_FORWARD (+1, Flow.forward, z -> x) or NFX_INVERSE (-1, Flow.inverse).
 *   - Numerical guards of the reference (NaN/Inf replacement, clamps) are part of the contract
 *     and reproduced exactly.
 */
#ifndef NFX_H
#define NFX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 3: the log_prob workspace (nfx_gauss_workspace_bytes) may hold anything on entry — the
 * fused epilogues' last workgroup finishes the float64 sums in the same launch, and its arrival
 * word carries a fixed tag: a word without it (garbage, a fill, zeros, another allocation's data)
 * is claimed once instead of added to (ABI 2 required a zero-filled workspace); nfx_made_affine_backward / nfx_made_seq_backward / nfx_made_backward_weights
 * return NFX_EUNSUPPORTED above nfx_made_backward_max_batch(d, H) (callers split the batch). */
#define NFX_ABI_VERSION 3

#define NFX_OK 0
#define NFX_EINVAL (-1)
#define NFX_EUNSUPPORTED (-2)
#define NFX_ELAUNCH (-3)

#define NFX_FORWARD 1
#define NFX_INVERSE (-1)

/* MADE-affine variants (nfx_made_affine). */
#define NFX_MAF_INVERSE 0 /* MaskedAutoregressiveFlow.inverse  (density, parallel)   */
#define NFX_IAF_FORWARD 1 /* InverseAutoregressiveFlow.forward (sampling, parallel)  */
#define NFX_MAF_FORWARD 2 /* MaskedAutoregressiveFlow.forward  (sampling, sequential) */
#define NFX_IAF_INVERSE 3 /* InverseAutoregressiveFlow.inverse (density, sequential)  */

/*
 * Raw (unpacked) parameters of one conditioner MLP, exactly as the reference nn.Modules
 * hold them (device pointers, nn.Linear layout [out, in]). A NULL bias means zero bias;
 * a NULL mask means dense; a NULL bn_w[i] means no BatchNorm after hidden layer i.
 * Used by the *_pack entry points, which fold BatchNorm (eval, running stats) and masks into
 * the MFMA operand layout the kernels read (see DESIGN.md "HBM/LDS layout").
 */
typedef struct NfxMlpRaw {
    const float* w[4];
    const float* b[4];
    const float* mask[4];
    const float* bn_w[3];
    const float* bn_b[3];
    const float* bn_rm[3];
    const float* bn_rv[3];
    float bn_eps;
    int n_layers;
} NfxMlpRaw;

int nfx_abi_version(void);
const char* nfx_last_error(void);
/* The name of the last kernel this thread launched (e.g. "made_seqp_kernel"); "" before any.
 * Profiling aid: which kernel of a family an entry point dispatched to. */
const char* nfx_last_kernel(void);
/* Test hook: overwrite the LDS of every CU with the 32-bit pattern `bits` (tests poison LDS
 * before a kernel to show it never reads LDS it did not write). */
int nfx_debug_fill_lds(uint32_t bits, void* stream);

/* ---------------------------------------------------------------------------------------
 * Affine coupling — CouplingLayer (src/flows/coupling/coupling_layer.py:5-111).
 *   forward  replaces coupling_layer.py:40-68, inverse replaces coupling_layer.py:70-96.
 * s_net / b_net: Linear(d,H) -> BN(H) -> ReLU -> Linear(H,H) -> BN(H) -> ReLU -> Linear(H,d)
 * (coupling_layer.py:18-35); BatchNorm is folded with its running statistics (eval mode).
 * mask: [d] fp32 0/1 (the layer's `mask` buffer).
 * ------------------------------------------------------------------------------------- */
size_t nfx_affine_packed_floats(int d, int H);
int nfx_affine_pack(const NfxMlpRaw* s_net, const NfxMlpRaw* b_net, const float* mask, int d,
                    int H, float* packed, void* stream);
int nfx_affine_coupling(const float* packed, const float* in, float* out, float* log_det,
                        int64_t B, int d, int H, int direction, int accumulate, void* stream);
/* Inverse + fused log_prob epilogue (the last layer of an inverse chain): also writes
 * logp[i] = -0.5*(fp32(d log 2pi) + sum_j out[i,j]^2) + log_det[i] and sums[2] as
 * nfx_gauss_logprob does; `workspace` holds nfx_gauss_workspace_bytes(B) bytes. */
int nfx_affine_coupling_logprob(const float* packed, const float* in, float* out, float* log_det,
                                float* logp, double* sums, void* workspace, int64_t B, int d,
                                int H, int accumulate, void* stream);
/* Which affine-coupling kernel runs: the streaming one (a wave per 64-sample chunk, weights
 * in LDS) or the small-batch one (a workgroup per 32 samples, the conditioner split across
 * 2*HT waves). Both compute the same function (output-layer sums associated differently,
 * within fp32 rounding). NFX_AFFINE_AUTO (default, or $NFX_AFFINE_POLICY) picks by an
 * occupancy cost model. policy >= 0 sets it and returns the previous policy; a negative value
 * only reads it. Process-wide; host-only (no GPU call). */
#define NFX_AFFINE_AUTO 0
#define NFX_AFFINE_STREAMING 1
#define NFX_AFFINE_SMALL 2
int nfx_affine_kernel_policy(int policy);

/* A whole chain of affine coupling layers in ONE launch (eval mode; NormalizingFlowModel /
 * RealNVP / SequentialFlow of CouplingLayers without between-layer BatchNorm): packs[l] is
 * layer l's image from nfx_affine_pack (all layers the same d in {2, 4, 8} and H <= 128),
 * n_layers <= 64. direction +1 runs layers 0 .. n-1 (forward), -1 runs n-1 .. 0 (inverse).
 * The per-layer arithmetic is nfx_affine_coupling's small-batch kernel (bit-identical to the
 * per-layer calls with policy NFX_AFFINE_SMALL); rows and the running log-det stay in LDS
 * between layers. log_det: written (accumulate = 0) or added to, as a chain of per-layer calls
 * would. `packs` is a HOST array of device pointers. The _logprob variant (inverse only) also
 * writes logp and the float64 [sum, count] partials like nfx_affine_coupling_logprob
 * (workspace: nfx_gauss_workspace_bytes(B)).
 * Two layouts: up to 64k rows (or under policy NFX_AFFINE_SMALL) the small-batch one above; beyond
 * (or under NFX_AFFINE_STREAMING) the streaming one for H <= 64 (csrc/nfx_affine_schain.hip: one
 * workgroup per CU carries its rows through every layer, the per-layer arithmetic of the
 * streaming nfx_affine_coupling kernel, bit-identical to those per-layer calls; the next layer's
 * weights are DMA'd into LDS while the current layer runs). NFX_EUNSUPPORTED when neither takes
 * (B, d, H): nfx_affine_chain_supported tells beforehand (host-only, no GPU call; it depends on
 * the current kernel policy). */
int nfx_affine_chain_supported(int64_t B, int d, int H);
int nfx_affine_chain(const float* const* packs, int n_layers, const float* in, float* out,
                     float* log_det, int64_t B, int d, int H, int direction, int accumulate,
                     void* stream);
int nfx_affine_chain_logprob(const float* const* packs, int n_layers, const float* in, float* out,
                             float* log_det, float* logp, double* sums, void* workspace, int64_t B,
                             int d, int H, int accumulate, void* stream);
/* The sampling pass with its base draw fused in (Flow.sample, src/flows/flow/flow.py:40-54; the
 * reference's throughput loop plots/_common.py:264-274): z ~ N(0, I) drawn on the device
 * (Philox4x32-10 keyed by `seed`, counter = (sample, offset); Box-Muller), then the forward chain,
 * in ONE launch of the small-batch chain (B up to 64k rows at d = 2; NFX_EUNSUPPORTED above).
 * rng_state: device uint64[2] = {counter offset, arrival count}, zero-filled once; every launch
 * reads the offset and its last workgroup advances it, so repeated launches (and replays of a
 * captured graph) draw fresh values. z (may be NULL) receives the draws, x = forward(z) bit for bit
 * as nfx_affine_chain would give for that z, log_det written. */
int nfx_affine_chain_sample(const float* const* packs, int n_layers, uint64_t seed, uint64_t* rng_state,
                            float* z, float* x, float* log_det, int64_t B, int d, int H, void* stream);

/* ---------------------------------------------------------------------------------------
 * Rational-quadratic spline coupling — SplineCouplingLayer
 * (src/flows/spline/spline_coupling_layer.py:6-323): forward :96-137, inverse :139-180,
 * spline core _rational_quadratic_spline :182-309, param net :56-62 (no BatchNorm).
 * rescale: 0 = data_min/data_max None (identity, :78-94); 1 = scalar rescale with
 * data_min/data_max given as fp32 scalars.
 * ------------------------------------------------------------------------------------- */
size_t nfx_spline_packed_floats(int d, int H, int K);
int nfx_spline_pack(const NfxMlpRaw* param_net, const float* mask, int d, int H, int K,
                    float* packed, void* stream);
int nfx_spline_coupling(const float* packed, const float* in, float* out, float* log_det,
                        int64_t B, int d, int H, int K, float bound, float min_bin_width,
                        float min_bin_height, float min_derivative, int rescale,
                        float data_min, float data_max, int direction, int accumulate,
                        void* stream);
/* Inverse + fused log_prob epilogue (see nfx_affine_coupling_logprob). */
int nfx_spline_coupling_logprob(const float* packed, const float* in, float* out, float* log_det,
                                float* logp, double* sums, void* workspace, int64_t B, int d,
                                int H, int K, float bound, float min_bin_width,
                                float min_bin_height, float min_derivative, int rescale,
                                float data_min, float data_max, int accumulate, void* stream);

/* A whole chain of SplineCouplingLayers in ONE launch (eval mode; NormalizingFlowModel /
 * RealNVPSpline, spline_coupling_layer.py:96-180 chained by normalizing_flow_model.py:40-65):
 * packs[l] = layer l's nfx_spline_pack image (a HOST array of device pointers), every layer
 * d = 2 with the same H <= 64, K, bound and minimums, no data_min/data_max rescale; n_layers <= 64.
 * direction +1 runs layers 0 .. n-1, -1 runs n-1 .. 0. One workgroup per CU carries its rows and
 * running log-det in LDS through every layer (csrc/nfx_spline_schain_kernel.h) with the per-layer
 * kernel's arithmetic: bit-identical to the per-layer nfx_spline_coupling calls. The _logprob
 * variant (inverse only) adds the Gaussian log-density and float64 [sum, count] as
 * nfx_spline_coupling_logprob. nfx_spline_chain_supported: host-only check of (B, d, H, K). */
int nfx_spline_chain_supported(int64_t B, int d, int H, int K);
int nfx_spline_chain(const float* const* packs, int n_layers, const float* in, float* out, float* log_det,
                     int64_t B, int d, int H, int K, float bound, float min_bin_width, float min_bin_height,
                     float min_derivative, int direction, int accumulate, void* stream);
int nfx_spline_chain_logprob(const float* const* packs, int n_layers, const float* in, float* out,
                             float* log_det, float* logp, double* sums, void* workspace, int64_t B, int d,
                             int H, int K, float bound, float min_bin_width, float min_bin_height,
                             float min_derivative, int accumulate, void* stream);
/* The sampling pass of a d = 2 spline chain (RealNVPSpline.forward on z ~ N(0, I)) with the base
 * draw fused in, as nfx_affine_chain_sample (same generator, same rng_state semantics). */
int nfx_spline_chain_sample(const float* const* packs, int n_layers, uint64_t seed, uint64_t* rng_state,
                            float* z, float* x, float* log_det, int64_t B, int d, int H, int K, float bound,
                            float min_bin_width, float min_bin_height, float min_derivative, void* stream);

/* ---------------------------------------------------------------------------------------
 * Unit-interval RQ spline — rational_quadratic_spline
 * (src/flows/spline/rational_quadratic_spline.py:4-104). Elementwise over N inputs with
 * per-input unnormalised widths/heights [N,K] and derivatives [N,K-1]; epsilon is forced to
 * 1e-6 exactly as the reference does (:19).
 * ------------------------------------------------------------------------------------- */
int nfx_rqs_unit(const float* in, const float* widths, const float* heights,
                 const float* derivatives, float* out, float* log_det, int64_t N, int K,
                 float min_bin_width, float min_bin_height, float min_derivative, int inverse,
                 void* stream);
/* Its adjoint (autograd of the same function, torch semantics: clamps pass the gradient on
 * their closed range, bin selection carries none): grad_out, grad_log_det [N] in; grad_in [N],
 * grad_widths / grad_heights [N,K], grad_derivatives [N,K-1] out (overwritten). */
int nfx_rqs_unit_backward(const float* in, const float* widths, const float* heights,
                          const float* derivatives, const float* grad_out, const float* grad_log_det,
                          float* grad_in, float* grad_widths, float* grad_heights, float* grad_derivatives,
                          int64_t N, int K, float min_bin_width, float min_bin_height, float min_derivative,
                          int inverse, void* stream);

/* ---------------------------------------------------------------------------------------
 * ARQS — autoregressive unit-interval RQ spline flow (src/flows/spline/arqs.py:7-114):
 * forward replaces arqs.py:44-80, inverse replaces arqs.py:82-114. One launch runs the
 * reference's d sequential steps (MADE on the partial output vector, view(B, d, 3K-1) row i,
 * rational_quadratic_spline of column i). made: the conditioner MADE(d, H, 3K-1) — its four
 * MaskedLinear layers with masks (and eval BatchNorm when use_batch_norm). H <= 128,
 * 2 <= K <= 11. rescale: 0 = data_min/data_max None; 1 = scalar rescale (x - data_min) /
 * (data_max - data_min) in fp32 with fp32(data_max - data_min) from the double difference.
 * ------------------------------------------------------------------------------------- */
size_t nfx_arqs_packed_floats(int d, int H, int K);
int nfx_arqs_pack(const NfxMlpRaw* made, int d, int H, int K, float* packed, void* stream);
int nfx_arqs(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d,
             int H, int K, float min_bin_width, float min_bin_height, float min_derivative,
             int rescale, double data_min, double data_max, int direction, int accumulate,
             void* stream);

/* ---------------------------------------------------------------------------------------
 * MADE-masked autoregressive affine flows — MADE (src/flows/autoregressive/made.py:6-140),
 * MaskedLinear (masked_linear.py:4-18), MaskedAutoregressiveFlow
 * (masked_autoregressive_flow.py:18-78), InverseAutoregressiveFlow
 * (inverse_autoregressive_flow.py:30-103). net: 4 masked layers, output order [mu | alpha].
 * variant: NFX_MAF_INVERSE / NFX_IAF_FORWARD (parallel, MFMA) or
 *          NFX_MAF_FORWARD / NFX_IAF_INVERSE (sequential over d).
 * Shapes: d <= 4096, H <= 256 (NFX_EUNSUPPORTED beyond).
 * ------------------------------------------------------------------------------------- */
size_t nfx_made_packed_floats(int d, int H);
int nfx_made_pack(const NfxMlpRaw* net, int d, int H, float* packed, void* stream);
/* nfx_made_pack in two parts: the parallel directions' image (+ degree tables and structural-zero
 * extents), then — required before an NFX_MAF_FORWARD / NFX_IAF_INVERSE nfx_made_affine(_logprob)
 * call on the buffer — the sequential directions' rank-ordered image and chunk schedule.
 * nfx_made_pack = both. */
int nfx_made_pack_parallel(const NfxMlpRaw* net, int d, int H, float* packed, void* stream);
int nfx_made_pack_sequential(int d, int H, float* packed, void* stream);
int nfx_made_affine(const float* packed, const float* in, float* out, float* log_det,
                    int64_t B, int d, int H, int variant, int accumulate, void* stream);
/* Density direction + fused log_prob epilogue (see nfx_affine_coupling_logprob):
 * NFX_MAF_INVERSE with d <= 64 or H <= 64 (and H <= 128), NFX_IAF_INVERSE (sequential) with H <= 64;
 * NFX_EUNSUPPORTED otherwise (use nfx_gauss_logprob after nfx_made_affine). */
/* Which kernel runs the SEQUENTIAL MADE directions (NFX_MAF_FORWARD, NFX_IAF_INVERSE) at
 * H <= 64: the segment-parallel one (16 lanes per sample, 4 samples per wave) or the
 * wave-per-sample one (64 lanes per sample: a ~4x shorter dependent chain per sample, for
 * small batches / strong scaling). Same function (mu/alpha dot products associated
 * differently, within fp32 rounding). NFX_MADE_SEQ_AUTO (default, or $NFX_MADE_SEQ_POLICY)
 * takes the wave-per-sample kernel up to 8 samples per CU (2,048 on 256 CUs), the segment kernel
 * above. policy >= 0 sets it and returns the previous one; negative reads.
 * Process-wide; host-only. */
#define NFX_MADE_SEQ_AUTO 0
#define NFX_MADE_SEQ_SEGMENT 1
#define NFX_MADE_SEQ_WAVE 2
/* NFX_MADE_SEQ_PUSH: the wave-per-sample PUSH kernel (made_seqp_kernel, d <= 1024): every step's
 * (mu, alpha) accumulated in registers as units complete, the completing unit's layer-1 sum formed
 * once; falls back to the wave kernel outside d <= 1024. */
#define NFX_MADE_SEQ_PUSH 3
int nfx_made_seq_policy(int policy);
int nfx_made_affine_logprob(const float* packed, const float* in, float* out, float* log_det,
                            float* logp, double* sums, void* workspace, int64_t B, int d, int H,
                            int variant, int accumulate, void* stream);

/* ---------------------------------------------------------------------------------------
 * Training: backward of the PARALLEL MADE directions under autograd —
 * MaskedAutoregressiveFlow.inverse (masked_autoregressive_flow.py:18-44, the density-training
 * direction; variant NFX_MAF_INVERSE) and InverseAutoregressiveFlow.forward
 * (inverse_autoregressive_flow.py:30-63; NFX_IAF_FORWARD) — for d <= 4096, H <= 128 and no
 * BatchNorm (NFX_EUNSUPPORTED otherwise).
 * nfx_made_pack_backward adds the transposed weight tiles to a packed image built by
 * nfx_made_pack (same buffer). nfx_made_affine_backward recomputes the layer and writes
 *   grad_in [B, d]  = dL/dx
 *   factors [3d + 6H + 4][P], feature-major rows (P = nfx_made_factor_pitch(B)):
 *     [δμ | δα] (2d) | δ3 | δ2 | δ1 (H each) | h3, 1 | h2, 1 | h1, 1 (H + 1 each) | x, 1 (d + 1)
 * from grad_out = dL/dz [B, d] and grad_log_det = dL/dlog_det [B]. The parameter gradients
 * are contractions over the sample dimension (nfx_made_backward_weights): dW4 = [δμ;δα]·h3ᵀ,
 * dW3 = δ3·h2ᵀ, dW2 = δ2·h1ᵀ, dW1 = δ1·xᵀ (each ⊙ its MADE mask), db = row sums of δ.
 * `factors` holds nfx_made_backward_factor_floats(B, d, H) floats.
 * ------------------------------------------------------------------------------------- */
int nfx_made_pack_backward(const NfxMlpRaw* net, int d, int H, float* packed, void* stream);
size_t nfx_made_backward_factor_floats(int64_t B, int d, int H);
/* Largest B one nfx_made_affine_backward / nfx_made_seq_backward / nfx_made_backward_weights
 * call accepts (the factor rows use 32-bit buffer offsets); larger batches are split by the
 * caller (the gradients are sums over samples). Above it the calls return NFX_EUNSUPPORTED. */
int64_t nfx_made_backward_max_batch(int d, int H);
int nfx_made_affine_backward(const float* packed, const float* in, const float* grad_out,
                             const float* grad_log_det, float* grad_in, float* factors, int64_t B,
                             int d, int H, int variant, void* stream);

/* MADE parameter gradients from the factors above (both MAF and IAF backward kernels write this
 * layout, rows of pitch nfx_made_factor_pitch(B) = B): fp32 MFMA contractions
 * over the sample dimension, reduced in float64 in a fixed order (deterministic), written to
 * `grads` in MADE.parameters() order — net.0.weight [H,d], net.0.bias [H], net.2.weight [H,H],
 * net.2.bias, net.4.weight, net.4.bias, net.6.weight [2d,H], net.6.bias [2d] — each weight
 * gradient multiplied by its mask (masks[4]: the MaskedLinear `mask` buffers, device, row-major;
 * the gradient of F.linear(a, W * mask, b), masked_linear.py:14-18). `grads` holds
 * nfx_made_param_floats(d, H) floats, `workspace` nfx_made_wgrad_workspace_bytes(B, d, H) bytes.
 * Replaces the autograd weight-gradient GEMMs of made.py:81-134. */
/* Backward of the SEQUENTIAL directions (NFX_IAF_INVERSE: inverse_autoregressive_flow.py:65-103,
 * the IAF density direction; NFX_MAF_FORWARD: masked_autoregressive_flow.py:46-78) for
 * d <= 4096, H <= 128, no BatchNorm: the d MADE calls of the reference are differentiated as one
 * forward recompute + one reverse sweep per sample (a triangular adjoint solve). Writes grad_in
 * and the same factor layout (X1 = the MADE input zs), so the parameter gradients are again
 * nfx_made_backward_weights. */
int nfx_made_seq_backward(const float* packed, const float* in, const float* grad_out,
                          const float* grad_log_det, float* grad_in, float* factors, int64_t B,
                          int d, int H, int variant, void* stream);
int64_t nfx_made_factor_pitch(int64_t B);
size_t nfx_made_param_floats(int d, int H);
size_t nfx_made_wgrad_workspace_bytes(int64_t B, int d, int H);
int nfx_made_backward_weights(const float* factors, int64_t B, int d, int H,
                              const float* const* masks, float* grads, void* workspace,
                              void* stream);

/* ---------------------------------------------------------------------------------------
 * Training: backward of SplineCouplingLayer.forward/inverse
 * (spline_coupling_layer.py:96-309 under autograd) in one fused kernel: the param MLP
 * recomputed on MFMA, the rational-quadratic spline's adjoint per transformed element (softmax,
 * knot cumsum with pinned ends, softplus, gather, RQ map / citardauq inverse, every clamp and
 * NaN/Inf guard as autograd treats it), the data-gradient chain through the MLP and the weight
 * gradients as contractions over the sample dimension. d <= 8, H <= 64, K <= 11, no data_min/
 * data_max rescale, and at most 2 (H <= 32) / 1 (H <= 64) transformed dimensions
 * (NFX_EUNSUPPORTED otherwise). packed: nfx_spline_pack_backward image; grads: fp32, the
 * layer's parameters() order (param_net.0.weight, .0.bias, .2.weight, .2.bias, .4.weight,
 * .4.bias); workspace: nfx_spline_backward_workspace_bytes(B, d, H, K) bytes.
 * ------------------------------------------------------------------------------------- */
size_t nfx_spline_backward_packed_floats(int d, int H, int K);
size_t nfx_spline_backward_param_floats(int d, int H, int K);
size_t nfx_spline_backward_workspace_bytes(int64_t B, int d, int H, int K);
int nfx_spline_pack_backward(const NfxMlpRaw* net, const float* mask, int d, int H, int K,
                             float* packed, void* stream);
int nfx_spline_coupling_backward(const float* packed, const float* mask, const float* in,
                                 const float* grad_out, const float* grad_log_det, float* grad_in,
                                 float* grads, void* workspace, int64_t B, int d, int H, int K,
                                 int n_transformed, float bound, float min_bin_width,
                                 float min_bin_height, float min_derivative, int direction,
                                 void* stream);

/* ---------------------------------------------------------------------------------------
 * Training (SURVEY.md §8(f) items 1 + 2): CouplingLayer in TRAIN mode — BatchNorm1d with
 * batch statistics (coupling_layer.py:18-35 under model.train(); the reference's training
 * loops README.md:107-117, plots/_common.py:194-211) — and its backward, for d <= 8, H <= 64
 * (NFX_EUNSUPPORTED otherwise). Replaces the autograd graph of coupling_layer.py:40-96.
 * Statistics are float64 triples stats[2 nets][Hp][3] = (n, mean, M2), Hp = 32*ceil(H/32),
 * so data-parallel ranks can merge them exactly (SyncBN); BatchNorm normalises with
 * var = M2/n and updates running_var with M2/(n-1) (momentum as given).
 * One layer's step (the caller orders them on one stream):
 *   nfx_affine_train_pack(stats1 = stats2 = NULL)  -> tpack (identity BatchNorm)
 *   nfx_affine_train_stats(layer 1)                -> stats1      [SyncBN: merge over ranks]
 *   nfx_affine_train_pack(stats1, NULL)            -> tpack
 *   nfx_affine_train_stats(layer 2)                -> stats2      [SyncBN: merge over ranks]
 *   nfx_affine_train_pack(stats1, stats2, epack)   -> tpack + eval-layout pack epack
 *   nfx_affine_coupling(epack, ...)                -> (y, log_det) of the train-mode layer
 *   nfx_affine_train_update_running                -> BatchNorm running statistics [4 BNs:
 *                                                     s_net.1, s_net.4, b_net.1, b_net.4]
 * backward, from grad_out = dL/dy [B,d] and grad_log_det [B]:
 *   nfx_affine_train_backward(stage 1, 2, 3)       -> G (float64 sums; stage-1/-2 BatchNorm
 *                                                     sums G[0:4Hp] and the stage-2 block are
 *                                                     all-reduced between stages under SyncBN)
 *                                                     and grad_in [B,d]
 *   nfx_affine_train_assemble                      -> fp32 parameter gradients in the layer's
 *                                                     parameters() order (s_net then b_net)
 * `workspace` holds nfx_affine_train_workspace_bytes(B, d, H) bytes and must be the same buffer
 * for stages 2 and 3 of one backward.
 * ------------------------------------------------------------------------------------- */
size_t nfx_affine_train_pack_floats(int d, int H);
size_t nfx_affine_train_stats_doubles(int H);
size_t nfx_affine_train_grad_doubles(int d, int H);
size_t nfx_affine_train_param_floats(int d, int H);
size_t nfx_affine_train_workspace_bytes(int64_t B, int d, int H);
int nfx_affine_train_pack(const NfxMlpRaw* s_net, const NfxMlpRaw* b_net, const float* mask,
                          const double* stats1, const double* stats2, int d, int H, float* tpack,
                          float* epack, void* stream);
int nfx_affine_train_stats(const float* tpack, const float* in, int64_t B, int d, int H, int layer,
                           double* stats, void* workspace, void* stream);
int nfx_affine_train_update_running(const double* stats1, const double* stats2,
                                    float* const* running_mean, float* const* running_var, int H,
                                    double momentum, void* stream);
/* The same, also adding 1 to the 4 BatchNorms' num_batches_tracked (int64 counters). */
int nfx_affine_train_update_running_counted(const double* stats1, const double* stats2,
                                            float* const* running_mean, float* const* running_var,
                                            int64_t* const* num_batches_tracked, int H,
                                            double momentum, void* stream);
int nfx_affine_train_backward(const float* tpack, const float* in, const float* grad_out,
                              const float* grad_log_det, float* grad_in, int64_t B, int d, int H,
                              int direction, int stage, const double* stats2, double* G,
                              void* workspace, void* stream);
int nfx_affine_train_assemble(const double* G, const double* stats1, const double* stats2, int d,
                              int H, float eps, float* grads, void* stream);
/* Kept activations (H <= 64): nfx_affine_train_stats_keep(layer 2, keep) also writes the raw
 * layer-2 pre-activations h2 = W2 a1 + b2 of both nets into `keep` (nfx_affine_train_keep_floats
 * floats, 512 B per sample at H = 64), and nfx_affine_train_backward_keep(stage 1 or 2, keep)
 * reads them instead of recomputing layers 1-2 (keep = NULL: the plain entry points). */
size_t nfx_affine_train_keep_floats(int64_t B, int d, int H);
int nfx_affine_train_stats_keep(const float* tpack, const float* in, int64_t B, int d, int H,
                                int layer, double* stats, void* workspace, float* keep,
                                void* stream);
int nfx_affine_train_backward_keep(const float* tpack, const float* in, const float* grad_out,
                                   const float* grad_log_det, float* grad_in, int64_t B, int d,
                                   int H, int direction, int stage, const double* stats2,
                                   double* G, void* workspace, const float* keep, void* stream);
/* The layer's (y, log_det) from the kept pre-activations, tpack folded with both statistics:
 * replaces nfx_affine_coupling(epack, ...) in a forward that kept them. */
int nfx_affine_train_output(const float* tpack, const float* in, const float* keep, float* out,
                            float* log_det, int64_t B, int d, int H, int direction, void* stream);
/* Eval-mode CouplingLayer under autograd (coupling_layer.py:40-96 with model.eval(): BatchNorm
 * normalises with its RUNNING statistics, which are buffers, so nothing couples the samples).
 * Same kernels: nfx_affine_eval_stats writes triples (-1, running_mean, -running_var) for the 4
 * BatchNorms (s_net.1, s_net.4, b_net.1, b_net.4); nfx_affine_train_pack(stats1, stats2) folds
 * them exactly like eval BatchNorm; nfx_affine_train_backward(stage 1..3) and
 * nfx_affine_train_assemble then give dL/dx and every parameter gradient (gamma/beta included)
 * with the batch-statistics terms of the BatchNorm backward dropped (n < 0). */
int nfx_affine_eval_stats(float* const* running_mean, float* const* running_var, int H,
                          double* stats1, double* stats2, void* stream);

/* ---------------------------------------------------------------------------------------
 * Gaussian base log-density + NLL partial sums — the log_prob glue of the callers
 * (Flow.log_prob src/flows/flow/flow.py:56-73; README.md:113-114; src/utils.py:39-55):
 *   logp[i] = -0.5 * (fp32(d*log(2*pi)) + sum_j z[i,j]^2) + log_det[i]
 * (torch.distributions.MultivariateNormal(0, I).log_prob(z) + log_det).
 * sums[0] = sum_i logp[i] in float64, sums[1] = B (as double). `workspace` must hold
 * nfx_gauss_workspace_bytes(B) bytes, of ANY content (ABI 3): every call that writes sums (this
 * one and the fused *_logprob epilogues) reduces the per-workgroup partials in its last workgroup;
 * the workspace's tagged arrival word is validated by the kernel itself (a foreign value is
 * replaced, not added to) and left clean, so one workspace serves any number of stream-ordered
 * calls (not two concurrent ones). nfx_gauss_workspace_init (optional, stream-ordered, graph-
 * capturable) writes the clean word up front; without it the first call on an uninitialised
 * workspace spends one compare-and-swap round per early workgroup. logp may be NULL (NLL-only).
 * ------------------------------------------------------------------------------------- */
size_t nfx_gauss_workspace_bytes(int64_t B);
int nfx_gauss_workspace_init(void* workspace, void* stream);
int nfx_gauss_logprob(const float* z, const float* log_det, float* logp, double* sums,
                      void* workspace, int64_t B, int d, void* stream);
/* Its adjoint (training: loss = -mean log p): grad_z[i, j] = -z[i, j] * grad_logp[i],
 * grad_log_det[i] = grad_logp[i] (autograd of the expression above). */
int nfx_gauss_logprob_backward(const float* z, const float* grad_logp, float* grad_z, float* grad_log_det,
                               int64_t B, int d, void* stream);

/* ---------------------------------------------------------------------------------------
 * Between-layer BatchNorm of NormalizingFlowModel(batch_norm_between_layers=True)
 * (src/models/normalizing_flow_model.py:67-128), an invertible per-feature affine with the
 * RUNNING statistics and a batch-constant log-det c = sum_j log|g_j| - 0.5 log(rv_j + eps):
 *   nfx_flowbn_apply   forward  out = (in - rm)/sqrt(rv + eps)*g + b, log_det[i] += c
 *                      (replaces _apply_batch_norm + _batch_norm_log_det_jacobian, :35-44);
 *                      inverse  out = (in - b)/g*sqrt(rv + eps) + rm, log_det[i] -= c (:55-60).
 *                      d <= 1024.
 * Train mode (forward direction, :74-79), before the apply:
 *   nfx_flowbn_moments        stats[d][3] = float64 (n, mean, M2) of the batch per feature
 *                             (SyncBN: merge the triples over ranks before the update)
 *   nfx_flowbn_update_running running = running*(1 - momentum) + momentum*batch (biased var)
 * Autograd of one apply w.r.t. the input and (weight, bias) — the running statistics are
 * buffers — from grad_out [B,d] and grad_log_det [B] (either may be NULL = zero):
 *   nfx_flowbn_backward       grad_in [B,d], grad_gamma [d], grad_beta [d]
 * `workspace` holds nfx_flowbn_workspace_bytes(B, d) bytes.
 * ------------------------------------------------------------------------------------- */
size_t nfx_flowbn_workspace_bytes(int64_t B, int d);
int nfx_flowbn_apply(const float* in, float* out, float* log_det, const float* gamma, const float* beta,
                     const float* running_mean, const float* running_var, float eps, int64_t B, int d,
                     int direction, void* stream);
int nfx_flowbn_moments(const float* x, int64_t B, int d, double* stats, void* workspace, void* stream);
int nfx_flowbn_update_running(const double* stats, float* running_mean, float* running_var,
                              double momentum, int d, void* stream);
int nfx_flowbn_backward(const float* in, const float* grad_out, const float* grad_log_det, float* grad_in,
                        const float* gamma, const float* beta, const float* running_mean,
                        const float* running_var, float eps, float* grad_gamma, float* grad_beta,
                        int64_t B, int d, int direction, void* workspace, void* stream);


/* ---------------------------------------------------------------------------------------
 * Any-shape path (csrc/nfx_generic.hip): the conditioner MLP of a layer whose shape is beyond
 * the fused kernel families, one nn.Linear at a time on fp32 MFMA, plus the spline coupling's
 * element math. Row-major fp32 device buffers; w is an nn.Linear weight [N][K] (out x in).
 * ------------------------------------------------------------------------------------- */
/* y[M][N] = act(((x[M][K] o in_scale[K]) (w o wmask)^T + b) o post_scale + post_shift): one
 * nn.Linear / MaskedLinear (wmask: its 0/1 mask, weight * mask as masked_linear.py:17) with an
 * optional per-feature affine after it (an eval-mode BatchNorm1d: post_scale = gamma/sqrt(rv+eps),
 * post_shift = beta - rm * post_scale) and ReLU when relu = 1. in_scale (e.g. the coupling mask:
 * Linear(x * mask)), wmask, b and the post affine may be NULL. Replaces the reference's
 * conditioner nn.Sequential one Linear (+ BatchNorm + ReLU) at a time. */
int nfx_linear_forward(const float* x, const float* w, const float* wmask, const float* b, const float* in_scale,
                       const float* post_scale, const float* post_shift, float* y, int64_t M, int K, int N,
                       int relu, void* stream);
/* gx[M][K] (+)= ((gy[M][N] (w o wmask)) o out_scale[K]), kept only where act[M][K] > 0 when act
 * is given (the ReLU backward of the layer feeding this Linear): autograd's input gradient of
 * nn.Linear. accumulate = 1 adds into gx. */
int nfx_linear_backward_data(const float* gy, const float* w, const float* wmask, const float* act,
                             const float* out_scale, float* gx, int64_t M, int N, int K, int accumulate, void* stream);
/* gw[N][K] = (gy^T (x o in_scale)) o wmask, gb[N] = sum over rows of gy (gb may be NULL):
 * autograd's weight and bias gradients of nn.Linear / MaskedLinear, split over the batch into a
 * workspace of nfx_linear_workspace_bytes(M, N, K) bytes and summed in a fixed order. */
size_t nfx_linear_workspace_bytes(int64_t M, int N, int K);
int nfx_linear_backward_weight(const float* gy, const float* x, const float* in_scale, const float* wmask, float* gw,
                               float* gb, int64_t M, int N, int K, void* workspace, void* stream);
/* MADE affine flows' element math for any (d, H) (the conditioner output params [B][2d] =
 * [mu | alpha] from nfx_linear_*): nfx_made_elem_forward — the parallel directions
 * (NFX_MAF_INVERSE: masked_autoregressive_flow.py:18-44, NFX_IAF_FORWARD:
 * inverse_autoregressive_flow.py:30-63) incl. guards and log-det clamp; nfx_made_elem_step —
 * step i of a sequential direction (NFX_MAF_FORWARD :46-78, NFX_IAF_INVERSE :65-103) on the
 * running vector `work` [B][d] (zeros at i = 0) and log-det `work_ld` [B] (zeros), then
 * nfx_made_elem_finish — the final guards and clamp into y / log_det (written or accumulated);
 * nfx_made_elem_backward — the adjoint of the parallel element map: gparams [B][2d] =
 * (dL/dmu, dL/dalpha) and gx the direct dL/dx term (gy / gld may be NULL). */
int nfx_made_elem_forward(const float* x, const float* params, float* y, float* log_det, int64_t B, int d,
                          int variant, int accumulate, void* stream);
int nfx_made_elem_step(const float* x, const float* params, float* work, float* work_ld, int64_t B, int d, int i,
                       int variant, void* stream);
int nfx_made_elem_finish(const float* x, const float* work, const float* work_ld, float* y, float* log_det,
                         int64_t B, int d, int variant, int accumulate, void* stream);
int nfx_made_elem_backward(const float* x, const float* params, const float* gy, const float* gld, float* gparams,
                           float* gx, int64_t B, int d, int variant, void* stream);
/* Adjoint pieces of a sequential direction (autograd through the reference's d MADE calls),
 * at the finished raw vector `work` and params = MADE(work): mode 0 writes out [B][d] = the
 * output guard's share of gy; mode 1 out [B][2d] = dL/dparams for the total adjoint lam [B][d];
 * mode 2 out [B][d] = dL/dx. The caller iterates lam = (mode 0) + MADE-input-VJP(mode 1) d times
 * (the Jacobian is strictly triangular), then takes the weight gradients from mode 1. */
int nfx_made_elem_seq_backward(const float* x, const float* params, const float* work, const float* lam,
                               const float* gy, const float* gld, float* out, int64_t B, int d, int variant, int mode,
                               void* stream);
/* Train-mode BatchNorm in the MADE of a sequential direction: each of the reference's d calls
 * normalises with the batch statistics of its own partial vector, so the backward runs call by
 * call. nfx_made_elem_seq_step_backward: step i's adjoint from lam [B][d] (column i final):
 * grad_params [B][2d] = call i's (dL/dmu_i, dL/dalpha_i) in row i and zeros elsewhere, grad_in
 * column i = dL/dx_i; params = call i's MADE output, work / work_ld = the forward's raw vector and
 * running log-det (the clamp decision). nfx_made_elem_prefix: out = work with columns >= i zeroed
 * (call i's conditioner input). */
int nfx_made_elem_seq_step_backward(const float* x, const float* params, const float* work, const float* work_ld,
                                    const float* lam, const float* grad_out, const float* grad_log_det,
                                    float* grad_params, float* grad_in, int64_t B, int d, int i, int variant,
                                    void* stream);
int nfx_made_elem_prefix(const float* work, float* out, int64_t B, int d, int i, void* stream);
/* CouplingLayer element math for any (d, H) (coupling_layer.py:40-96): s_raw, b_raw [B][d] are
 * the raw s_net / b_net outputs; forward (+1) or inverse (-1) affine map with the clamps, guards
 * and log-det; the backward gives dL/ds_raw, dL/db_raw and the direct dL/dx term. */
int nfx_affine_elem_forward(const float* x, const float* s_raw, const float* b_raw, const float* mask, float* y,
                            float* log_det, int64_t B, int d, int direction, int accumulate, void* stream);
int nfx_affine_elem_backward(const float* x, const float* s_raw, const float* b_raw, const float* mask,
                             const float* gy, const float* gld, float* gs, float* gb, float* gx, int64_t B, int d,
                             int direction, void* stream);
/* A conditioner BatchNorm1d at any width N: nfx_bn_prepare turns batch moments (stats: float64
 * (n, mean, M2) per feature from nfx_flowbn_moments, SyncBN-merged; running statistics updated
 * with the unbiased variance when update_running) or, with stats = NULL, the running statistics
 * into mean / invstd / scale = gamma invstd / shift = beta - mean scale (BN(z) = z scale + shift);
 * nfx_bn_apply_relu h = relu(z scale + shift); the backward takes g = dL/dBN-output (ReLU mask
 * applied): nfx_bn_backward_sums sums [2][N] = (sum g = dL/dbeta, sum g xhat = dL/dgamma) in
 * float64 (workspace nfx_bn_workspace_bytes(M, N)); nfx_bn_backward_apply dL/dz (train: the
 * batch-statistics terms with the global sample count *count, a device float64 — the n of the
 * merged moments triple). */
int nfx_bn_prepare(const double* stats, const float* gamma, const float* beta, float* running_mean,
                   float* running_var, double eps, double momentum, int update_running, int N, float* mean,
                   float* invstd, float* scale, float* shift, void* stream);
int nfx_bn_apply_relu(const float* z, const float* scale, const float* shift, float* h, int64_t M, int N,
                      void* stream);
size_t nfx_bn_workspace_bytes(int64_t M, int N);
int nfx_bn_backward_sums(const float* g, const float* z, const float* mean, const float* invstd, double* sums,
                         int64_t M, int N, void* workspace, void* stream);
int nfx_bn_backward_apply(const float* g, const float* z, const float* mean, const float* invstd,
                          const float* gamma, const double* sums, const double* count, int train, float* gz,
                          int64_t M, int N, void* stream);
/* ARQS at any (d, H) and its backward (arqs.py:44-114, rational_quadratic_spline.py:4-104):
 * one sequential step i on params = MADE(state) [B][d (3K-1)] (viewed [B, d, 3K-1] like the
 * reference). mode 0: state[:, i] = spline(xr[:, i]) with params row i, log_det += its log-det;
 * mode 1 (reverse): with lam [B][d] = dL/d(state after step i) and gld the log-det gradient,
 * gparams row i = dL/d(params row i) (row i + 1 zeroed), gx[:, i] = dL/dxr[:, i], lam[:, i] = 0
 * (the caller adds the MADE-input VJP of gparams into lam); mode 2: state[:, i] = 0.
 * 2 <= K <= 11, data_min/data_max None. */
int nfx_arqs_step(const float* xr, const float* params, float* state, float* log_det, const float* gld, float* lam,
                  float* gparams, float* gx, int64_t B, int d, int K, int i, int direction, int mode,
                  float min_bin_width, float min_bin_height, float min_derivative, void* stream);
/* ARQS data_min / data_max bounds on the any-shape path (arqs.py:28-42), element-wise with
 * bounds = device [2][d] = data_min | data_max - data_min (scalar bounds broadcast), rounded as the
 * reference's expressions: mode 0 out = (in - lo) / w (to the unit interval), 1 out = in * w + lo
 * (back), and their adjoints 2 out = in / w, 3 out = in * w. */
int nfx_arqs_bounds(const float* in, const float* bounds, float* out, int64_t B, int d, int mode, void* stream);
/* SplineCouplingLayer element math for any d (spline_coupling_layer.py:96-180 with the spline
 * of :182-309): params [B][d][3K-1] = param_net output; dims with mask == 0 go through the RQ
 * spline (forward: direction +1, inverse: -1), the rest pass through; layer guards and the
 * log-det (sum over transformed dims, guarded; written or added with accumulate). 2 <= K <= 11,
 * data_min/data_max None. */
int nfx_spline_elem_forward(const float* x, const float* params, const float* mask, float* y, float* log_det,
                            int64_t B, int d, int K, float bound, float min_bin_width, float min_bin_height,
                            float min_derivative, int direction, int accumulate, void* stream);
/* Its adjoint: gparams [B][d][3K-1] = dL/dparams (zero for conditioning dims) and gx [B][d] =
 * the direct dL/dx term (the conditioner's contribution is added by nfx_linear_backward_data
 * with out_scale = mask). gy / gld (dL/dy, dL/dlog_det) may be NULL (zero). */
int nfx_spline_elem_backward(const float* x, const float* params, const float* mask, const float* gy,
                             const float* gld, float* gparams, float* gx, int64_t B, int d, int K, float bound,
                             float min_bin_width, float min_bin_height, float min_derivative, int direction,
                             void* stream);
/* The same with data_min / data_max bounds (spline_coupling_layer.py:78-94, scalar or
 * per-dimension): bounds = device [3][d] = data_min | 2B/(data_max - data_min) |
 * (data_max - data_min)/(2B) per dimension, rounded as the reference's expressions round them;
 * x is the raw input (the spline runs on to (x - lo) - B, its outputs map back, and the
 * backward's dL/dx includes both scales). nfx_spline_rescale writes xr = to (x - lo) - B, the
 * conditioner's input (times the mask in nfx_linear_forward). */
int nfx_spline_elem_forward_bounded(const float* x, const float* params, const float* mask, const float* bounds,
                                    float* y, float* log_det, int64_t B, int d, int K, float bound,
                                    float min_bin_width, float min_bin_height, float min_derivative, int direction,
                                    int accumulate, void* stream);
int nfx_spline_elem_backward_bounded(const float* x, const float* params, const float* mask, const float* bounds,
                                     const float* gy, const float* gld, float* gparams, float* gx, int64_t B, int d,
                                     int K, float bound, float min_bin_width, float min_bin_height,
                                     float min_derivative, int direction, void* stream);
int nfx_spline_rescale(const float* x, const float* bounds, float* xr, int64_t B, int d, float bound, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NFX_H */
