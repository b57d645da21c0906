#!/usr/bin/env python3
"""A/B of SimpleUNet's edge convolutions (the 65-channel input 3x3 and the 64 -> 65 ``out`` 1x1): the framework's
padded kernel paths (ops/conv.py ``_bias_conv3x3_padded_ok`` / ``_BiasConv1x1Fn``) vs MIOpen / CK, in-step through
``bench.py --layout unet-ddp``.  ``--arm miopen`` patches the two predicates off before the bench runs; run the arms
interleaved in one gpurun call (cdna_hip_programming.md rule 24).

    python benchmarks/probes/unet_edge_ab.py --arm dph|miopen [bench.py args ...]
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    args = sys.argv[1:]
    arm = "dph"
    if args[:1] == ["--arm"]:
        arm, args = args[1], args[2:]
    if arm == "miopen":
        from distributed_pytorch_hpc_amd.ops import conv

        conv._bias_conv3x3_padded_ok = lambda *a: False
        conv._bias_conv1x1_ok = lambda *a: False
    sys.argv = [os.path.join(ROOT, "bench.py"), "--layout", "unet-ddp"] + args
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
