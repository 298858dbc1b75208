/*
 * npd.h -- C ABI of libnpd.so, the MI355X-native batch Polar/PAC decoding hot path.
 *
 * The reference (hebbarashwin/neural_polar_decoder) is pure Python/PyTorch with no FFI; its
 * "operator API" for this path is the Python method surface of PolarCode / PAC / RNN_decoder /
 * convNet.  Each entry point below replaces one of those methods (cited per function); the Python
 * mirror in neural_polar_decoder_amd/ binds them with ctypes.
 *
 * Conventions
 *   - All tensor pointers are DEVICE pointers owned by the caller (e.g. torch tensors' data_ptr()),
 *     row-major fp32 unless stated: y/x (B,N), msg/msg_hat (B,K), exactly the reference's layouts.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  Every call is
 *     stream-ordered and asynchronous; none allocates or synchronises, so calls can be captured
 *     into a hipGraph.
 *   - Handles (npd_code, npd_gru, npd_conv) are immutable after creation: concurrent use from
 *     several host threads on distinct streams is safe.  A handle is bound to the device that was
 *     current when it was created.
 *   - Return value: 0 = success; > 0 = hipError_t passthrough; < 0 = argument error (NPD_E*).
 *     npd_last_error() returns a thread-local description of the last failure.  Nothing aborts.
 *   - Random numbers: Philox4x32-10, counter = (block, stream, codeword index), key = seed, so
 *     results are independent of how codewords are sharded over launches or GPUs.
 */
#ifndef NPD_H_
#define NPD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NPD_ABI_VERSION 1

#define NPD_OK 0
#define NPD_EINVAL (-1)   /* bad argument (null pointer, size, unsupported N/K) */
#define NPD_ENOTSUP (-2)  /* configuration not compiled in */
#define NPD_ENOMEM (-3)   /* host allocation failed */

typedef struct npd_code npd_code; /* a Polar or PAC code: N, K, info set, frozen prior, PAC taps */
typedef struct npd_gru npd_gru;   /* a CRISP GRU decoder's weights, repacked for the kernel */
typedef struct npd_conv npd_conv; /* a convNet decoder's weights, repacked for the kernel */

int npd_abi_version(void);
const char* npd_last_error(void);
/* number of visible HIP devices (0 when none); never fails */
int npd_device_count(void);

/* ---------------------------------------------------------------------------------- codes */
/*
 * Create a code.  Replaces PolarCode.__init__ (polar.py:66-117) and PAC.__init__/rate_profiler
 * (pac_code.py:97-174): the caller passes the sorted information set it computed (rate profiles
 * are host logic).  pac_g == 0 -> Polar code; otherwise the PAC convolution polynomial (91 in the
 * reference; its top bit must be set).  infty = the Polar frozen-leaf prior (polar.py:66, default
 * 1000), ignored for PAC (pac_sc_decode applies no prior).  4 <= N <= 256, N a power of two.
 */
int npd_code_create(int N, int K, const int32_t* info_sorted, int pac_g, float infty, npd_code** out);
int npd_code_destroy(npd_code* code);

/* ---------------------------------------------------------------------------------- encode */
/*
 * x = encode(msg).  Polar: PolarCode.encode_plotkin (polar.py:128-148) -- u = ones, u[info] = msg,
 * butterfly left *= right for d = 0..n-1 (bit-exact for any fp32 input, same product order).
 * PAC: PAC.pac_encode (pac_code.py:220-224) -- rate profile, conv pre-transform, rate-1 Plotkin.
 */
int npd_encode(const npd_code* code, const float* msg, float* x, int64_t B, void* stream);

/* ---------------------------------------------------------------------------------- channel */
/*
 * y = x + fl32(sigma) * n, n ~ N(0,1) from Philox stream (seed, snr_index), codeword index
 * cw_offset + b.  Replaces PolarCode.channel / PAC.channel (polar.py:201-207, pac_code.py:226-231).
 * N % 4 == 0.
 */
int npd_awgn(const float* x, float* y, int64_t B, int N, float sigma, uint64_t seed, uint32_t snr_index,
             uint64_t cw_offset, void* stream);

/*
 * Fused Monte-Carlo data generation for codewords cw_offset .. cw_offset+B-1: msg bits from Philox
 * (seed), encode (Polar or PAC), AWGN at (sigma, snr_index).  Any of msg/x may be NULL; y required.
 * Equivalent to msg = 1-2*bits; x = encode(msg); y = channel(x, snr) in the reference eval loops
 * (run_models.py:318-323, rnn_all.py:842-847).
 */
int npd_mc_generate(const npd_code* code, float* msg, float* x, float* y, int64_t B, float sigma, uint64_t seed,
                    uint32_t snr_index, uint64_t cw_offset, void* stream);

/* ---------------------------------------------------------------------------------- SC decode */
/*
 * Successive-cancellation min-sum decoding, one codeword per lane.
 * Polar: PolarCode.sc_decode_new (polar.py:465-484): LLR = llr_scale * y with
 *   llr_scale = fl32(2/sigma^2); f = sign(a)sign(b)min(|a|,|b|) (utils.py:272-275); g = u*a + b;
 *   leaf = L + infty on frozen positions; u = sign(leaf).  Outputs: leaf_llr (B,N) [optional],
 *   msg_hat = u[:, info] (B,K) [optional].  u_hat must be NULL.
 * PAC: PAC.pac_sc_decode (pac_code.py:534-573): same tree, no prior, conv-state leaf rule.
 *   Outputs: leaf_llr (B,N), msg_hat = v_hat[:, info] (B,K), u_hat (B,N); each optional.
 * gt (B,N) optional genie (use_gt polar.py:480 / use_gt_codeword pac_code.py:548-555), else NULL.
 * Decisions and leaf LLRs are bit-exact with the reference (fp32, same operation order).
 */
int npd_sc_decode(const npd_code* code, const float* y, float llr_scale, float* leaf_llr, float* msg_hat,
                  float* u_hat, const float* gt, int64_t B, void* stream);

/*
 * Monte-Carlo SC decode with fused error counting: decodes y (B,N) of codewords
 * cw_offset .. cw_offset+B-1 whose messages are the Philox message stream of `seed` (as written
 * by npd_mc_generate), writes msg_hat (B,K) if non-NULL, and adds {bit errors, block errors} to
 * counters[0..1] (device uint64, not reset).  Error semantics of errors_ber/errors_bler
 * (utils.py:17-51): a decision of 0 counts as an error.
 */
int npd_sc_decode_mc(const npd_code* code, const float* y, float llr_scale, float* msg_hat, uint64_t seed,
                     uint64_t cw_offset, int64_t B, unsigned long long* counters, void* stream);

/*
 * Exact log-sum-exp SC, PolarCode.sc_decode(noisy_code, snr) (polar.py:209-279): check node =
 * log_sum_avoid_zero_NaN (utils.py:295-397), g = u*a + b, frozen leaves decided +1 (no prior),
 * information leaves sign(L) (hard_decision != 0, args.hard_decision) or tanh(L/2) (hard_decision == 0,
 * the reference's default).  Outputs (each optional): msg_hat = sign(decoded_bits)[:, info] (B,K) and
 * u_bits = decoded_bits (B,N).  Polar codes, N <= 256.  exp/log/tanh are the device libm, so values
 * agree with torch's CPU path to a few ulp (decisions except on near-zero LLRs).
 */
int npd_sc_decode_lse(const npd_code* code, const float* y, float llr_scale, int hard_decision, float* msg_hat,
                      float* u_bits, int64_t B, void* stream);

/*
 * Soft-output SC, PolarCode.sc_decode_soft(noisy_code, snr, priors) (polar.py:281-358): LSE check
 * nodes, leaf L^ = clamp(L + prior, -1000, 1000), right-child input LSE(L^_left, L_a) + L_b, nodes
 * return [LSE(L^_u, L^_v), L^_v]; frozen positions get no special treatment (priors carry them).
 * priors: HOST array of N floats or NULL (zeros).  Outputs as npd_sc_decode_lse.  4 <= N <= 256, y
 * 16-byte aligned.
 */
int npd_sc_decode_soft(const npd_code* code, const float* y, float llr_scale, int hard_decision, const float* priors,
                       float* msg_hat, float* u_bits, int64_t B, void* stream);

/*
 * PolarCode.sc_decode_soft_new(corrupted_codewords, snr, priors) (polar.py:485-607: updateLLR_soft,
 * partial_decode_soft, updatePartialSums_soft): SC whose partial sums are LLRs ("soft partial sums",
 * [a, b] -> [LSE(a, b), b] per stage) -- the decode_soft recursion above -- with the leaf stored as
 * clamp(L + prior, +-1000) + prior.  Outputs msg_hat (B,K) = sign(stored leaf)[:, info] (the reference's
 * return value) and optionally u_hat (B,N) = sign of every stored leaf.  priors (N floats, host) or NULL
 * (zeros: frozen positions are decided like information positions, as in the reference).  Polar codes,
 * 4 <= N <= 256, y 16-byte aligned.
 */
int npd_sc_decode_soft_new(const npd_code* code, const float* y, float llr_scale, const float* priors, float* msg_hat,
                           float* u_hat, int64_t B, void* stream);

/* ---------------------------------------------------------------------------------- SC-List decode */
/*
 * Successive-cancellation list decoding, PolarCode.scl_decode(y, snr, L, use_CRC=False)
 * (polar.py:793-876) with pruneLists (polar.py:777-791): min-sum SC per path (no frozen prior in the
 * LLRs), path metric += |leaf| on a frozen leaf with sign(leaf) != 1 and on the flipped branch of an
 * information leaf; survivors = torch.topk's choice (ties resolved exactly as std::nth_element, see
 * npd_list_prune_select) in list order; final path = the first minimum of ||encode(u) - y||^2.
 * Polar codes, 8 <= N <= 256, 1 <= list_size <= 8, y 16-byte aligned.  Outputs: msg_hat (B,K) and
 * u_hat (B,N) of the chosen path, each optional.  scl_decode's leaf-LLR output equals
 * npd_sc_decode(..., gt = u_hat) (a genie pass reproduces the chosen path's LLRs bit for bit).
 * Decisions are bit-exact with the reference except when two list candidates' fp32 distances differ
 * only by summation order (torch's vectorised sum vs a sequential one here).
 */
int npd_scl_decode(const npd_code* code, const float* y, float llr_scale, int list_size, float* msg_hat,
                   float* u_hat, int64_t B, void* stream);
/* Monte-Carlo SC-List decode with fused error counting (semantics of npd_sc_decode_mc). */
int npd_scl_decode_mc(const npd_code* code, const float* y, float llr_scale, int list_size, float* msg_hat,
                      uint64_t seed, uint64_t cw_offset, int64_t B, unsigned long long* counters, void* stream);
/*
 * Host utility (no GPU): the survivor set of pruneLists for n <= 16 candidates whose negated metrics
 * are neg_metrics[0..n) in list order, keeping `keep` -- bit c of *mask_out set iff candidate c
 * survives.  The same code runs inside the SCL kernel when metrics tie across the boundary.
 */
int npd_list_prune_select(const float* neg_metrics, int n, int keep, uint32_t* mask_out);

/*
 * A whole SNR sweep of npd_sc_decode_mc in one launch: y is (n_snr, B, N) -- the received words of
 * the same codewords cw_offset .. cw_offset+B-1 at n_snr SNR points (the reference's per-SNR loop,
 * run_models.py:318-371), llr_scale a HOST array of n_snr scales, msg_hat (n_snr, B, K) or NULL,
 * counters (n_snr, 2).  1 <= n_snr <= 16.  Same results as n_snr separate npd_sc_decode_mc calls.
 */
int npd_sc_decode_mc_sweep(const npd_code* code, int n_snr, const float* y, const float* llr_scale, float* msg_hat,
                           uint64_t seed, uint64_t cw_offset, int64_t B, unsigned long long* counters, void* stream);

/*
 * The Monte-Carlo step in one launch, y never stored: for each of the n_snr segments s and codeword
 * cw_offset .. cw_offset+B-1, the message (Philox message stream of `seed`), its codeword and the
 * received word (noise stream snr_index0 + s, sigma[s]) are generated in registers exactly as
 * npd_mc_generate writes them, SC-decoded with llr_scale[s] and counted into counters (n_snr, 2)
 * (and msg_hat (n_snr, B, K) if non-NULL).  Equal, count for count, to npd_mc_generate (snr_index =
 * snr_index0 + s) followed by npd_sc_decode_mc_sweep.  sigma and llr_scale are HOST arrays.  Polar
 * codes with 8 <= N <= 64 (NPD_ENOTSUP otherwise).  Replaces the generate/decode/count body of the
 * reference's eval loops (run_models.py:318-337, rnn_all.py:842-856) for the SC decoder.
 */
int npd_sc_mc_sweep_fused(const npd_code* code, int n_snr, const float* sigma, const float* llr_scale,
                          uint32_t snr_index0, uint64_t seed, uint64_t cw_offset, int64_t B, float* msg_hat,
                          unsigned long long* counters, void* stream);

/* ---------------------------------------------------------------------------------- counters */
/*
 * counters[0] += #(round(ref) != round(hat)), counters[1] += #rows with any such element, over
 * (B,K) fp32 arrays.  Replaces errors_ber / errors_bler's counting (utils.py:17-51) with device
 * uint64 counters (no host sync per batch).
 */
int npd_count_errors(const float* ref, const float* hat, int64_t B, int K, unsigned long long* counters,
                     void* stream);

/*
 * As npd_count_errors, comparing ref (B,K) with columns cols[0..K) (HOST array, each < W) of hat (B,W):
 * the reference's `errors_ber(msg, decoded[:, info])` (rnn_all.py:874-879, run_models.py:333-337)
 * without materialising the gathered (B,K) copy.  K <= 256.
 */
int npd_count_errors_cols(const float* ref, const float* hat, int64_t B, int K, int W, const int32_t* cols,
                          unsigned long long* counters, void* stream);

/*
 * errors_ber(ref, hat, mask) with an integer mask (utils.py:17-25; the loops pass torch.ones(...).long(),
 * run_models.py:325-341): counters[0] += sum(mask * (round(ref) != round(hat))), counters[1] += sum(mask),
 * over (B,K) arrays (mask int64).  errors_ber = counters[0] / counters[1], decided on the device (no host
 * read of the mask).
 */
int npd_count_errors_masked(const float* ref, const float* hat, const int64_t* mask, int64_t B, int K,
                            unsigned long long* counters, void* stream);

/* ---------------------------------------------------------------------------------- CRISP GRU */
/*
 * Create a GRU decoder from an RNN_Model state dict (rnn_all.py:294-398): nn.GRU(input_size, F,
 * layers, batch_first) + Linear(F, 1), decoding_type y_input without the y-MLP.
 * weights: host fp32, packed per layer l = 0..layers-1 as
 *   weight_ih_l (3F, Din_l) | weight_hh_l (3F, F) | bias_ih_l (3F) | bias_hh_l (3F),
 * then linear.weight (F) | linear.bias (1); Din_0 = N + 2 (onehot) or N + 1, Din_l = F for l > 0.
 * precision: 0 = fp32 (default, exact fp32 FMA chains), 1 = bf16x3 split, 2 = bf16, 3 = fp16x3 split (hi + lo fp16
 * parts, three products per multiply, fp32 accumulation: held to the fp32 path's tolerance; F <= 64).
 */
int npd_gru_create(int N, int F, int layers, int onehot, const float* weights, int64_t n_weights, int precision,
                   npd_gru** out);
int npd_gru_destroy(npd_gru* gru);
/*
 * npd_gru_create for either cell of rnn_all.py:69 (--rnn_type GRU | LSTM): cell 0 = GRU (npd_gru_create), cell 1 =
 * LSTM (nn.LSTM, gates i, f, g, o; the same weight order with 4F gate rows: weight_ih_l (4F, Din_l) | weight_hh_l (4F, F)
 * | bias_ih_l (4F) | bias_hh_l (4F) per layer, then linear.weight | linear.bias).  LSTM: fp32 (precision 0), hidden
 * 32, 64, 128, 256 or 512, 1 or 2 layers (F = 512 with 2 layers: N <= 128, as the GRU), y_input decoding (npd_gru_decode) or
 * y_h0 decoding (npd_gru_decode_ex with y = NULL: h and c both start from h0, as get_h0 returns (x, x) for LSTM,
 * rnn_all.py:370-375); destroy with npd_gru_destroy.
 */
int npd_rnn_create(int cell, int N, int F, int layers, int onehot, const float* weights, int64_t n_weights, int precision,
                   npd_gru** out);
/*
 * npd_rnn_create with the reference's other output heads (rnn_all.py:317-343; forward rnn_all.py:387-398: decoded =
 * linear(layernorm(out))).  GRU cells, fp32 (precision 0), F 32 or 64 (gru_decode_kernel), unidirectional.
 *  - --use_layernorm: ln_weight / ln_bias (F, host) are nn.LayerNorm(F)'s gamma / beta, ln_eps its eps.  The affine part
 *    folds into the output Linear (w gamma, b + w . beta); the kernel normalises each step's top-layer state (two-pass
 *    mean and biased variance over the F units).  ln_weight = NULL: no LayerNorm.
 *  - --out_linear_depth > 1 (head_depth): linear = Linear(F, H), SELU, [Linear(H, H), SELU] x (depth - 2), Linear(H, 1)
 *    with H = head_hidden (the net's y_hidden_size, 1 .. 128); head_weights (host) = the Linear layers' weight and
 *    bias in order (W_0 (H, F), b_0 (H), ..., W_last (1, H), b_last (1)), n_head values; the last F + 1 values of
 *    `weights` (the depth-1 linear) are then ignored.  Each head layer is an fp32 MFMA GEMM per step inside the decode
 *    loop.  head_depth = 1: the plain Linear(F, 1) of `weights`.  Not combined with the LayerNorm.
 * ln_weight = NULL and head_depth = 1 is npd_rnn_create.
 */
int npd_rnn_create_ex(int cell, int N, int F, int layers, int onehot, const float* weights, int64_t n_weights,
                      int precision, const float* ln_weight, const float* ln_bias, float ln_eps, int head_depth,
                      int head_hidden, const float* head_weights, int64_t n_head, npd_gru** out);
/*
 * RNN_decoder.decode(net, False, y, gt) test branch (rnn_all.py:532-547): decoded (B,N) fp32, with
 * decoded[:, i] = sign(out_i) for i in the info set (is_info: N bytes, host) and 1 (or gt) else.
 * reverse: RNN_decoder reverse_order (rnn_all.py:414-416).  logits (B,N) optional: raw output at
 * every step.
 */
int npd_gru_decode(const npd_gru* gru, const float* y, const uint8_t* is_info, int reverse, const float* gt,
                   float* decoded, float* logits, int64_t B, void* stream);
/*
 * The same decode with an initial state and an optional y input -- decoding_type 'y_h0' (rnn_all.py:523-531):
 * hidden = net.get_h0(y), then every step's RNN input is onehot(previous decision) alone.  The handle is created
 * from weights whose weight_ih_l0 carries N zero columns before the one-hot / sign columns (the y_input layout with
 * the y part zero); y = NULL skips that projection.  h0: (B, F * layers) fp32 on the device, element f * layers + l =
 * layer l, hidden unit f -- get_h0's x before its reshape(-1, F, layers).permute(2, 0, 1) (rnn_all.py:362-375).
 * Precision 0, or the 16-codeword split kernel (F = 64, 2 layers, N % 32 == 0); y = NULL and h0 = NULL is an error.
 * LSTM handles take exactly one of y (y_input) and h0 (y_h0, both states start from it), fp32.
 */
int npd_gru_decode_ex(const npd_gru* gru, const float* y, const float* h0, const uint8_t* is_info, int reverse,
                      const float* gt, float* decoded, float* logits, int64_t B, void* stream);
/*
 * The eval loop's GRU half over an SNR sweep (rnn_all.py:853-880: at each SNR point decoded = RNN_decoder.decode(y_s),
 * then errors_ber / errors_bler(msg, decoded[:, info]), rnn_all.py:874-879, utils.py:17-51): y is (n_seg, B, N), one
 * segment of received words per SNR point; msg (B, K) the message bits of the B codewords (the same messages in every
 * segment: the Monte-Carlo driver's message stream is keyed by codeword, not SNR); cols (K, HOST) the decoded columns
 * compared with msg's columns.  counters (n_seg, 2) += [bit errors, block errors] of each segment -- equal, count for
 * count, to npd_gru_decode_ex + npd_count_errors_cols per segment.  decoded (n_seg, B, N) is optional for the
 * 16-codeword split kernel (F = 64, 2 layers, N % 32 == 0, precision != 0), which decodes and counts every segment in
 * ONE launch (errors counted in the decision epilogue, one atomic pair per wave and segment); other handles run one
 * decode + one count per segment and need decoded.  y_input decoding, no gt, no logits.
 */
int npd_gru_decode_count_sweep(const npd_gru* gru, int n_seg, const float* y, const uint8_t* is_info, int reverse,
                               const float* msg, int K, const int32_t* cols, float* decoded, int64_t B,
                               unsigned long long* counters, void* stream);
/*
 * One layer of RNN_Model.get_h0 / get_Fy (rnn_all.py:362-385): out (B, Nout) = act(x (B, K) W^T + bias), W (Nout, K)
 * row-major, all device fp32, k summed in order.  act: 0 linear, 1 relu, 2 selu, 3 elu, 4 tanh, 5 sigmoid
 * (RNN_Model.act, rnn_all.py:346-360).  get_h0 follows layer ii with act iff ii != y_depth (rnn_all.py:364-368): every
 * layer, the last included, when y_depth >= 2; all but the last when y_depth = 1 (two layers) -- the caller passes
 * act = 0 for that one layer.
 */
int npd_ymlp_layer(const float* x, const float* W, const float* bias, float* out, int64_t B, int K, int Nout, int act,
                   void* stream);

/* ---------------------------------------------------------------------------------- conv model */
/*
 * convNet (models.py:691-772) forward/decode.  weights: host fp32 in state_dict order
 * (layers1.0.weight, layers1.0.bias, ..., layersFin.4.bias, layer_norm.weight, layer_norm.bias).
 * embed = config.embed_dim (even), N = config.N = config.max_len.
 * precision: 0 = fp32 (exact fp32 FMA chains); 3 = fp16x3 (conv layers with cin > 1 and the Linear layers: hi + lo
 * fp16 operands on the fp16 MFMA, three products per multiply, fp32 accumulation, weights scaled by 2^SW per layer
 * and activations by 2^4 before the split; layer 0, epilogues and LayerNorm fp32).
 */
int npd_conv_create(int N, int embed, const float* weights, int64_t n_weights, int precision, npd_conv** out);
int npd_conv_destroy(npd_conv* conv);
/* logits (B,N) and/or decoded = sign(logits) (B,N); workspace sized by npd_conv_workspace_bytes */
int64_t npd_conv_workspace_bytes(const npd_conv* conv, int64_t B);
int npd_conv_forward(const npd_conv* conv, const float* y, float* logits, float* decoded, void* workspace,
                     int64_t B, void* stream);
/* As npd_conv_forward, and (if input4 != NULL) the intermediate activation convNet.forward also returns,
 * input4 = layers3(input3) + input3 (models.py:750, :767), channels-first (B, embed/2, N) fp32. */
int npd_conv_forward_ex(const npd_conv* conv, const float* y, float* logits, float* decoded, float* input4,
                        void* workspace, int64_t B, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NPD_H_ */
