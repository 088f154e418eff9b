#!/usr/bin/env python3
"""Reference-compatible entry point: ``python train.py [--batch-size N] [--epochs N] [--lr LR]
[--gamma M] [--no-cuda] [--dry-run] [--seed S] [--log-interval N] [--save-model]`` plus the
framework's extensions (see pytorch_distributed_training_example_amd/cli.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_distributed_training_example_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
