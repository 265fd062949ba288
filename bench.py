#!/usr/bin/env python3
"""Driver contract entry point: `python bench.py --gpus N --steps K --warmup W`.

Runs the headline UserBootstrap churn benchmark (see
bacchus_gpu_controller_amd/bench/harness.py) and prints one JSON line on rank 0.
Under torchrun each rank drives one GPU; the native binaries are built in-tree first.
"""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _ensure_built():
    # Build once (rank 0 / single process); other ranks wait for the artefacts.
    rank = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    marker = os.path.join(ROOT, "bin", "kube-lite")
    if rank == 0:
        from bacchus_gpu_controller_amd.utils.build import ensure_built

        # stdout carries exactly one JSON line: build chatter (ninja/hipcc are child
        # processes writing to fd 1) goes to stderr
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            ensure_built()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    else:
        import time

        for _ in range(600):
            if os.path.exists(marker):
                break
            time.sleep(0.5)


if __name__ == "__main__":
    _ensure_built()
    from bacchus_gpu_controller_amd.bench.harness import main

    sys.exit(main())
