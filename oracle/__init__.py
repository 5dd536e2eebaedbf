"""CPU oracle for the geometric message-passing hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain-PyTorch (CPU, fp32 or fp64) restatement of the reference's algorithm
(NW-JEFF/Geometric-Message-Passing; file:line citations in each module). It exists to *check*
the HIP product path and to provide the CPU baseline leg of bench.py. Only `tests/`,
`__graft_entry__.smoke()` and bench.py's `cpu_baseline` may import it; the product package
(`geometric-message-passing_amd/gmp_amd`) never does, and has no CPU fallback.

Pinning:
  * scatter / propagate / EGNN / GVP / radial: pinned against golden vectors produced by running
    the reference's own layer code (tests/golden/make_golden.py, stubbed plumbing imports).
  * e3nn-derived pieces (spherical harmonics, wigner_3j, FullyConnectedTensorProduct, o3.Linear,
    BatchNorm, Gate, U matrices / SymmetricContraction) and PyG SchNet: the third-party source is
    absent from the container and from /root/reference, so these are restated from the published
    algorithms of e3nn 0.5.1 / PyG 2.3.1 and checked by known-answer and equivariance tests only:
    **parity unpinned** for those rows.
"""
