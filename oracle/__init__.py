"""CPU oracle for the dense-depth training hot path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU (PyTorch/ATen CPU ops and numpy), the
reference algorithms of LuizGuzzo/Monocular_Depth_Estimation that the HIP
kernels of `monocular_depth_estimation_amd` replace.  Each function cites the
reference file:line it follows.

Rules:
  * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
    import this package, and only as the checker / the timed CPU baseline.
  * The product package never imports it; its ops raise on CPU tensors.

Pinning: the restatement is checked against golden fixtures captured by
importing the reference itself in the build container
(tests/golden/make_golden.py -> tests/golden/*.npz; see tests/test_oracle_golden.py).
The MobileNetV3-Large encoder (torchvision, absent here) is "parity unpinned".
"""
