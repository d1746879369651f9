"""ORACLE — test infrastructure only.

CPU restatement of jackperlo/onnx-rusty-inference-engine's fp32 op path (C, `ref_ops.c` +
`ref_engine.c`, built by `oracle/Makefile` into `oracle/liboracle.so`).  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this package, and only
as the checker / the CPU baseline.  The product (`onnx-rusty-inference-engine_amd/`) never
imports it.
"""
from .oracle import *  # noqa: F401,F403
