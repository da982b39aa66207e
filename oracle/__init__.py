"""CPU oracle for the pcseg hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in the product package (`3d-semantic-segmentation-benchmark_amd/pcseg`)
may import this package.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` use it, and only as the checker / the timed
CPU baseline -- never as the thing measured or shipped.

Parity pinning: the restatement in `ref_ops.py` is checked against golden
vectors captured from the reference itself (`tests/golden/make_golden.py`
imports /root/reference in the build container and writes `.npz` fixtures).
"""
