"""Process-wide switches, read from the environment ONCE (at import) instead of on every op call.

Round 2 read ``os.environ`` inside every convolution / BatchNorm call (28 ``PDT_*`` lookups per
conv, ``tools/host_overhead.py``: 9 ms of host time per ResNet-50 step, binding at the reference's
128 images per GPU). The hot path now reads plain attributes of ``SW``. Tests and A/B tools that
flip a switch inside one process set the variable and call ``SW.reload()`` (tests: the ``switch``
fixture in ``tests/conftest.py``).

Switch                      default      meaning
PDT_DISABLE_NATIVE          0            1: every op on its PyTorch reference path (stock baseline)
PDT_CONV1X1                 auto         1x1 conv backend: auto (measured table) | ours | gemm | miopen | off
PDT_CONV1X1_OURS            fwd,dgrad,wgrad  directions allowed on our MFMA kernels (conv1x1.hip, conv1x1_wgrad.hip)
PDT_CONV1X1_PREFER          fwd,bwd_data directions that take our GEMM regardless of the table ("none": table only)
PDT_CONV1X1_OVERRIDE        ""           per-shape decisions "dir,dtype,M,Ci,Co=algo;..." (A/B tools)
PDT_CONV1X1_TABLE           1            0: ignore tuning/conv1x1_gfx950.json
PDT_CONV1X1_DUMP            ""           write the decisions to this path at exit
PDT_CONV1X1_S2              1            stride-2 1x1 shortcut as gather + GEMM
PDT_CONV3X3                 ours         3x3 convs on our kernels (ours | miopen)
PDT_CONV3X3_WGRAD           ours         3x3 weight gradient on our kernel (ours | miopen)
PDT_CONV3X3_S2              ours         stride-2 3x3 convs on our kernels (ours | miopen)
PDT_CONV_STEM               ours         7x7 stem on our kernels (ours | miopen)
PDT_CONV_BN_STATS           1            BatchNorm statistics in conv epilogues
PDT_BN_BWD_STATS            1            BatchNorm backward reduction in dgrad epilogues
PDT_RES_MASKED              1            ReLU'd residual gradient handed over as (dy, mask)
PDT_STEM_BWD_FUSED          1            stem pool backward takes the BN backward reduction
PDT_STEM_BN_WGRAD           1            stem weight gradient applies the stem BN backward on load
PDT_STEM_POOL_WGRAD         1            ... and forms the max-pool gradient itself (pooled dy + codes): dz never in HBM
PDT_STRIDED_BSTATS          1            a transition block's conv1 data gradient adds the stride-2 shortcut's compact
                                         gradient AND takes the previous block's bn3 backward reduction in our
                                         GEMM's epilogue (vs hipBLASLt + scatter-add + a reduce pass)
PDT_GAP_NATIVE              1            ResNet global-average-pool gradient on our kernel, with the last bn3's
                                         backward reduction
PDT_STEM_BN_STATS           1            stem conv emits its BatchNorm's statistics (no reduce pass; W == 224)
PDT_WGRAD_SPLITK            1            split-K 1x1 weight gradients
PDT_SLICE_SUM               1            split-K partial sums on our slice_sum kernel
PDT_SUBSAMPLE_NATIVE        1            stride-2 gather / scatter-add kernels
PDT_LINEAR_SPLITK           1            split-K Linear weight gradients
PDT_FUSED_ADDLN             1            residual add fused into LayerNorm
PDT_EMBEDDING_NATIVE        1            GPT-2 token/position embedding on our kernels
PDT_BWD_FUSED               1            bottleneck conv3 + bn3 backward as one kernel (conv1x1_bwd_fused.hip):
                                         bn3's backward apply formed on load, conv3 dgrad + wgrad + bn2 reduction
PDT_BWD_FUSED_SHAPES        256x64       (Co x Ci) of the conv3s that take the fused backward ("256x64,512x128" adds
                                         layer 2: 0.9 % slower in-step since the branch-free conv1x1 epilogue,
                                         profiles/r5/ab_layer2_unfused.txt)
PDT_BWD_ALG                 2            bottleneck conv3 + bn3 backward (the shapes PDT_BWD_FUSED does not take) without
                                         bn3's apply pass: z = a W^T substituted into bn3's backward (ops/conv.py
                                         _bwd_alg, csrc/kernels/bn_alg.hip): one wgrad pass + one data-gradient GEMM;
                                         2: also bn3's backward reduction without reading z (sum-only producer)
PDT_Z3_VIRTUAL              0            (with PDT_BWD_ALG=2) a bottleneck conv3 output (bn3 input) is never written —
                                         statistics-only GEMM, bn3's apply as the GEMM again (APPLY epilogue): 1 every
                                         block; 2 only where that APPLY GEMM runs anyway (conv3 input channels <=
                                         PDT_BN_APPLY_GEMM_K: the skipped store is then pure gain)
PDT_ALG_GLO                 1            the ALG data gradient carries G = W^T diag(B) W as a bf16 hi + lo pair (a twice
                                         in K). 0 (hi only, K = C4 + CW + 32) ran +1.0 % but is NOT kept: the dropped
                                         lo half is a fixed matrix, so its error a (G - G_hi) is correlated with bn2's
                                         input and biases bn2's gamma gradient (10.5 % vs 4.6 % from fp32 in
                                         tests/test_conv1x1_ours_gpu.py::test_bottleneck_chain_takes_bn_backward_stats;
                                         profiles/r6/ab_alg_glo.txt)
PDT_BWD_ALG_MIN_M           50176        the ALG paths (conv3 and shortcut) only for convs with at least this many output
                                         pixels: their small per-block GEMMs cost ~30-60 us whatever the batch, more
                                         than the apply pass they remove on ResNet-50 layers 3-4 at 128 images/GPU
PDT_BWD_ALG_FIRST           1            the ALG backward also where PDT_BWD_FUSED would run (layer 1's conv3)
PDT_DS_ALG                  512          the ALG backward for a downsample block's shortcut conv + BN too, where the
                                         conv has <= this many input channels (0 = off): the shortcut BN's
                                         reduction and apply passes go; sum(g) comes from bn3's backward (same g)
PDT_BN2_DEFER               0            1: with PDT_BWD_FUSED, bn2's apply + ReLU deferred into conv3 (read on load
                                         in the forward GEMM, recomputed in the fused backward, which writes bn2's
                                         mask). Measured -0.2 %, and -2 % with PDT_BN_APPLY_GEMM_K (the relu(a x + b)
                                         operand transform then runs in both GEMM passes): off
PDT_SUB_OUT                 1            a ResNet stage's last BatchNorm apply also writes the stride-2 subsample the next
                                         stage's strided 1x1 shortcut reads (its gather pass does not run)
PDT_BN_APPLY_GEMM_K         0            a BatchNorm(+residual)+ReLU apply after a 1x1 conv with <= this many input
                                         channels runs as that conv's GEMM again with the apply epilogue (reads
                                         the conv input, C/4 channels, instead of its output; 0 = off). Round 4
                                         (256-channel GEMM tiles): 128 (layers 1-2) +0.7 % over off, 64 +0.2 % over
                                         128 (profiles/r4/ab_bn_apply_gemm.md). Round 6, with the ALG backward: 64
                                         is 0.4 % SLOWER than off (16,202-16,226 vs 16,265-16,287 img/s, same box,
                                         profiles/r6/ab_apply_gemm_r6.txt): the layer-1 APPLY GEMM runs at ~4 TB/s
                                         (906-1217 us) against the 5.4 TB/s apply pass
PDT_LINEAR_EPILOGUE         auto         Linear forward GEMMs (+bias, MLP fc1+bias+GELU) on our MFMA kernel (gemm.hip)
                                         per shape by measurement (tuning/linear_gfx950.json, else timed once);
                                         1 / 0: forced on / off
PDT_FP8_FUSED_GELU          1            fp8 MLPs: bias+GELU (and its backward) emit e4m3 + transpose directly
                                         (fp8.hip fp8_gelu_cast_kernel): no bf16 activation, no cast pass
PDT_FP8_WEIGHT_MULTI        1            fp8: every Linear weight cast in one launch per forward (fp8_cast_multi)
PDT_FP8_CAST_COLSUM         1            fp8: a Linear's output-gradient cast also yields its bias gradient
PDT_FP8_LN                  1            fp8: the add+LayerNorm in front of qkv / fc1 writes its output as e4m3 +
                                         transpose for that GEMM (layernorm.hip ln_fwd_fp8_kernel): no bf16 y
PDT_WGRAD_STREAM_M          0            conv weight gradients with <= this many output pixels run on a side
                                         stream, concurrent with their data gradient (0 = in-stream)
"""
from __future__ import annotations

import os


class _Switches:
    __slots__ = ("disable_native", "conv1x1", "conv1x1_ours", "conv1x1_prefer", "conv1x1_override",
                 "conv1x1_table", "conv1x1_dump", "conv1x1_s2", "conv3x3", "conv3x3_wgrad", "conv3x3_s2", "conv_stem",
                 "conv_bn_stats", "bn_bwd_stats", "res_masked", "stem_bwd_fused", "stem_bn_wgrad", "stem_bn_stats", "stem_pool_wgrad", "wgrad_splitk", "slice_sum",
                 "subsample_native", "linear_splitk", "fused_addln", "embedding_native", "linear_epilogue",
                 "bwd_fused", "bwd_fused_shapes", "bwd_alg", "alg_glo", "bwd_alg_min_m", "z3_virtual", "bwd_alg_first", "ds_alg", "bn2_defer", "bn_apply_gemm_k", "strided_bstats", "gap_native", "sub_out",
                 "fp8_fused_gelu", "fp8_weight_multi", "fp8_cast_colsum", "fp8_ln", "wgrad_stream_m")

    def __init__(self):
        self.reload()

    def reload(self) -> "_Switches":
        e = os.environ.get

        def on(name: str, default: str = "1") -> bool:
            return e(name, default) != "0"

        self.disable_native = e("PDT_DISABLE_NATIVE", "0") == "1"
        self.conv1x1 = e("PDT_CONV1X1", "auto")
        self.conv1x1_ours = tuple(e("PDT_CONV1X1_OURS", "fwd,dgrad,wgrad").split(","))
        # our GEMM for the 1x1 forward and data gradients of every shape (layers 3-4 included): on par
        # with hipBLASLt in-step (profiles/r5/ab_conv1x1_prefer.txt), and its epilogues take the BN work
        self.conv1x1_prefer = tuple(p for p in e("PDT_CONV1X1_PREFER", "fwd,bwd_data").split(",") if p)
        ov = e("PDT_CONV1X1_OVERRIDE", "")
        self.conv1x1_override = dict(p.split("=", 1) for p in ov.replace("+", ";").split(";") if "=" in p)
        self.conv1x1_table = on("PDT_CONV1X1_TABLE")
        self.conv1x1_dump = e("PDT_CONV1X1_DUMP") or None
        self.conv1x1_s2 = e("PDT_CONV1X1_S2", "1") == "1"
        self.conv3x3 = e("PDT_CONV3X3", "ours")
        self.conv3x3_wgrad = e("PDT_CONV3X3_WGRAD", "ours")
        self.conv3x3_s2 = e("PDT_CONV3X3_S2", "ours")
        self.conv_stem = e("PDT_CONV_STEM", "ours")
        self.conv_bn_stats = on("PDT_CONV_BN_STATS")
        self.bn_bwd_stats = on("PDT_BN_BWD_STATS")
        self.res_masked = on("PDT_RES_MASKED")
        self.stem_bwd_fused = on("PDT_STEM_BWD_FUSED")
        self.stem_bn_wgrad = on("PDT_STEM_BN_WGRAD")
        self.stem_bn_stats = on("PDT_STEM_BN_STATS")
        # the stem weight gradient forms the max-pool gradient itself from (pooled dy, winner codes):
        # the 1.6 GB pool-input gradient is neither written nor read back (conv_stem.hip POOL)
        self.stem_pool_wgrad = on("PDT_STEM_POOL_WGRAD")
        self.wgrad_splitk = on("PDT_WGRAD_SPLITK")
        self.slice_sum = on("PDT_SLICE_SUM")
        self.subsample_native = on("PDT_SUBSAMPLE_NATIVE")
        self.linear_splitk = on("PDT_LINEAR_SPLITK")
        self.fused_addln = on("PDT_FUSED_ADDLN")
        self.embedding_native = on("PDT_EMBEDDING_NATIVE")
        # "auto": per-shape measured choice between our GEMM and hipBLASLt (ops/linear.py _ours); "1" / "0": forced
        self.linear_epilogue = e("PDT_LINEAR_EPILOGUE", "auto")
        self.bwd_fused = on("PDT_BWD_FUSED")
        self.bwd_fused_shapes = tuple(tuple(int(v) for v in t.split("x")) for t in
                                      e("PDT_BWD_FUSED_SHAPES", "256x64").split(",") if "x" in t)
        # 0 off; 1: ALG backward; 2: also the producer of bn3's gradient skips reading bn3's input for the backward
        # reduction (sum-only epilogue) and the ALG pass completes it (ops/batchnorm.py _BNTrainFn.backward)
        self.bwd_alg = int(e("PDT_BWD_ALG", "2"))
        self.bwd_alg_min_m = int(e("PDT_BWD_ALG_MIN_M", "50176"))
        self.alg_glo = on("PDT_ALG_GLO", "1")
        # bottleneck conv3 on the ALG backward: z (bn3's input) never written — statistics-only GEMM, bn3 applied by
        # the GEMM again (APPLY epilogue); recomputed only on a fallback (ops/conv.py materialize_virtual)
        self.z3_virtual = int(e("PDT_Z3_VIRTUAL", "0"))
        # the ALG backward also for the conv3 shapes the fused kernel takes (ResNet-50 layer 1: 256x64)
        self.bwd_alg_first = on("PDT_BWD_ALG_FIRST", "1")
        # the ALG backward for the downsample shortcut conv + BN (input channels <= this; 0 = off)
        self.ds_alg = int(e("PDT_DS_ALG", "512"))
        self.bn2_defer = on("PDT_BN2_DEFER", "0")
        self.bn_apply_gemm_k = int(e("PDT_BN_APPLY_GEMM_K", "0"))
        self.strided_bstats = on("PDT_STRIDED_BSTATS")
        self.gap_native = on("PDT_GAP_NATIVE")
        self.sub_out = on("PDT_SUB_OUT")
        self.fp8_fused_gelu = on("PDT_FP8_FUSED_GELU")
        self.fp8_weight_multi = on("PDT_FP8_WEIGHT_MULTI")
        self.fp8_cast_colsum = on("PDT_FP8_CAST_COLSUM")
        self.fp8_ln = on("PDT_FP8_LN")
        # conv weight gradients of at most this many output pixels run on a side stream, concurrent
        # with their data gradient (0 = off): small-batch grids leave CUs idle (ops/conv.py _WgradFork)
        self.wgrad_stream_m = int(e("PDT_WGRAD_STREAM_M", "0"))
        return self


SW = _Switches()
