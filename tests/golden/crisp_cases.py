"""Trained CRISP fixture cases: code, GRU and curriculum (shared by gen_trained.py and train_crisp_gpu.py).

Curricula follow run_crisp.sh:2-16: rate profile 'rev_polar' (Polar) / 'rev_RM' (PAC) with --target_K the
final K, K + 1 per stage, --dec_train_snr 0, batch 4096, AdamW lr 1e-3, StepLR(2000, 0.95), teacher forcing
ratio 1, a long final stage.  Each stage is (K, steps, trainer): trainer "ref" = the reference's own
rnn_all.py, unmodified, on the CPU (gen_trained.py); "gpu" = train_crisp_gpu.py's restatement of the same
loop on one MI355X.  GPU stages come first; the final stage(s) always run the reference's own loop.
"""


def _cur(first_K, first_steps, target_K, per_stage, final_gpu, final_ref, who="gpu"):
    cur = [(first_K, first_steps, who)]
    cur += [(k, per_stage, who) for k in range(first_K + 1, target_K)]
    if final_gpu:
        cur.append((target_K, final_gpu, who))
    cur.append((target_K, final_ref, "ref"))
    return cur


_COMMON = dict(F=64, layers=2, snr_train=0.0, batch=4096, lr=1e-3, lr_decay=2000, lr_gamma=0.95,
               eval_snrs=[0.0, 2.0, 4.0], n_dec=4096, n_mc=1 << 20)

CASES = {
    # the reference's own loop (CPU) for K = 4 .. 16, then a long K = 16 stage on the GPU and a last stage of the
    # reference's loop (run_crisp.sh's final stage is 100k steps)
    "trained_crisp_32_16": dict(_COMMON, code="Polar", profile="rev_polar", N=32, K=16, seed_init=3216,
                                curriculum=_cur(4, 2000, 16, 1000, 0, 8000, who="ref") + [(16, 40000, "gpu"),
                                                                                         (16, 1000, "ref")],
                                ref_lr=1e-3, n_logit=512, n_sc=1 << 17, seed_dec=31, seed_mc=37),
    # K = 8 .. 32 on the GPU, easiest bits first (rate profile 'polar', run_rnn_e2h.sh's direction), then the
    # reference's loop at K = 32.  (The hard-first order of run_crisp.sh, kept below as trained_crisp_64_32_h2e, left
    # the hidden-64 net at BER 0.33-0.42 / BLER ~1 over 0-4 dB after 81k GPU steps: the 24 more reliable bits added
    # after K = 8 stayed near coin flips, 0.5 error on bits 38-58 even at 10 dB.)
    "trained_crisp_64_32": dict(_COMMON, code="Polar", profile="polar", N=64, K=32, seed_init=6433,
                                curriculum=_cur(8, 3000, 32, 1000, 10000, 1000), ref_lr=2e-4,
                                n_logit=256, n_sc=1 << 16, seed_dec=41, seed_mc=43),
    "trained_crisp_64_32_h2e": dict(_COMMON, code="Polar", profile="rev_polar", N=64, K=32, seed_init=6432,
                                    curriculum=_cur(8, 5000, 32, 2000, 30000, 1000), ref_lr=2e-4,
                                    n_logit=256, n_sc=1 << 16, seed_dec=41, seed_mc=43),
    # round 6: configs[2]'s code and width, Polar(64,32) hidden 64, on run_crisp.sh's full schedule --
    # rev_polar (hard first), 10000 steps at K = 8, 5000 per K + 1 stage, 100000 at K = 32 (225k GPU steps, HIP-graph
    # replayed steps), then the reference's rnn_all.py for the last stage
    "trained_crisp_64_32_full": dict(_COMMON, code="Polar", profile="rev_polar", N=64, K=32, seed_init=6434,
                                     curriculum=_cur(8, 10000, 32, 5000, 100000, 1000), ref_lr=2e-4,
                                     n_logit=256, n_sc=1 << 16, seed_dec=41, seed_mc=43),
    # round 6: run_crisp.sh's code at configs[2]'s width -- Polar(64,22) hidden 64 -- on the easy-first order ('polar')
    # with a long last stage, for a decoding net on the headline kernel's own length (N = 64).  NOT GENERATED: learned
    # through K = 16 and diverged in the K = 17 stage (profiles/round6/train_crisp_64_22_h64.txt)
    "trained_crisp_64_22": dict(_COMMON, code="Polar", profile="polar", N=64, K=22, seed_init=6423,
                                curriculum=_cur(8, 3000, 22, 2000, 20000, 20), ref_lr=2e-4,
                                n_logit=256, n_sc=1 << 16, seed_dec=79, seed_mc=83),
    # run_crisp.sh's own decoder: Polar(64,22), rate profile rev_polar (hard first), GRU hidden 512, 2 layers, onehot
    # y_input, K = 8 .. 22 with K + 1 per stage.  The script runs 10000 steps at K = 8, 5000 per later stage and 100000 at
    # K = 22 (175k steps); this case runs the same stage order on the GPU with shortened stages (a GPU-minute budget),
    # then the reference's rnn_all.py for the last stage.
    "trained_crisp_64_22_f512": dict(_COMMON, code="Polar", profile="rev_polar", N=64, K=22, F=512, seed_init=6422,
                                     curriculum=_cur(8, 6000, 22, 1500, 20000, 20), ref_lr=2e-4,
                                     n_logit=128, n_sc=1 << 14, n_dec=2048, n_mc=1 << 17, seed_dec=59, seed_mc=61),
    # round 6: a scaled-down PAC decoder for configs[3]'s code family (rnn_all.py:61 --code PAC, g = 91), PAC(32,16) at
    # configs[3]'s width (hidden 64): K = 4 .. 16 on the GPU, then the reference's own loop for a last short stage (as
    # trained_crisp_64_22_f512).  Hard first ('rev_RM') at AdamW lr 3e-4: at the reference's 1e-3 the hard-first order
    # (trained_pac_32_16_rev) learned through K = 10 (BLER 0.48 / 0.25 / 0.08 at 0 / 2 / 4 dB) and ended at BLER
    # 0.93-0.98 at K = 16, and the easy-first order ('RM', trained_pac_32_16_rm) diverged at K = 11
    # (profiles/round6/train_pac_32_16.txt; those runs used g = 91, a PAC code of pac_code.py but not the one rnn_all.py
    # trains at N = 32, so they are GPU-only curriculum experiments)
    # the PAC(32,16) attempts below all learned their codes through K = 10 and lost them after: the PAC fixture is the
    # standard PAC(32,10) 'RM' code (the easy-first order's own K = 10 set), trained to its K with a long last stage.
    # g = 53: rnn_all.py:231-232 fixes the convolution by N (53 at N = 32; 91 from N = 64), whatever --g says
    "trained_pac_32_10": dict(_COMMON, code="PAC", profile="RM", N=32, K=10, g=53, seed_init=3210,
                              curriculum=_cur(4, 3000, 10, 3000, 20000, 20), ref_lr=2e-4,
                              n_logit=512, n_sc=1 << 15, seed_dec=67, seed_mc=69),
    "trained_pac_32_16": dict(_COMMON, code="PAC", profile="rev_RM", N=32, K=16, seed_init=3219, lr=3e-4,
                              curriculum=_cur(4, 3000, 16, 3000, 30000, 20), ref_lr=2e-4,
                              n_logit=512, n_sc=1 << 15, seed_dec=71, seed_mc=73),
    "trained_pac_32_16_rm": dict(_COMMON, code="PAC", profile="RM", N=32, K=16, seed_init=3218,
                                 curriculum=_cur(4, 3000, 16, 3000, 30000, 20), ref_lr=2e-4,
                                 n_logit=512, n_sc=1 << 15, seed_dec=71, seed_mc=73),
    "trained_pac_32_16_rev": dict(_COMMON, code="PAC", profile="rev_RM", N=32, K=16, seed_init=3217,
                                  curriculum=_cur(4, 3000, 16, 1500, 30000, 20), ref_lr=2e-4,
                                  n_logit=512, n_sc=1 << 15, seed_dec=71, seed_mc=73),
    # PAC(128,64) (configs[3], rnn_all.py:61 --code PAC, rate profile 'RM' reversed = hard first) at the CRISP script's
    # own width (run_crisp.sh: --rnn_feature_size 512): K = 8 .. 64 on the GPU, then the reference's loop.  At hidden 64
    # the same curriculum stalled (per-bit BER 0.08-0.26 even at 10 dB by K = 12, in either bit order).  NOT GENERATED:
    # this F = 512 run learned through K = 28 (BLER 0.71 / 0.38 / 0.12 at 0 / 2 / 4 dB) and collapsed to coin flips by
    # K = 61 (BER 0.45-0.49) with 400-step stages (the reference runs 5000); DESIGN.md 2b
    "trained_pac_128_64_f512": dict(_COMMON, code="PAC", profile="rev_RM", N=128, K=64, F=512, seed_init=12866,
                                    curriculum=_cur(8, 2000, 64, 400, 10000, 20), ref_lr=2e-4,
                                    n_logit=64, n_sc=1 << 13, n_dec=4096, n_mc=1 << 16, seed_dec=47, seed_mc=53),
}
