"""CPU oracle for the SPEF inference hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference algorithm of every step of the path
(MobileNet-V2 + URSONet forward in float32, softmax / Markley quaternion average / position
soft-argmax decode, keypoint projection, EPnP) so the HIP path can be checked against it.

Rules (DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
    and only as the checker / the timed CPU baseline -- never as the product path.
  * The product package (``spef_amd``) never imports it; the product fails loudly if its HIP library
    is missing.
  * Pinning: ``tests/golden/make_golden.py`` runs the *reference itself* (imported read-only from
    /root/reference in the build container) and commits its outputs as ``tests/golden/*.npz``;
    ``tests/test_oracle_golden.py`` checks this oracle against them. EPnP has no reference runner
    (OpenCV absent): it is pinned by noise-free known-answer tests only -- see ``epnp_ref``.
"""
