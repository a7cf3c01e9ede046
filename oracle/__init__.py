"""TEST INFRASTRUCTURE ONLY — CPU oracle for the DeepHall VMC hot path.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker (or the timed CPU baseline), never as the thing measured
or shipped.  The product path (``deephall_amd``) never imports this package and
fails loudly when its HIP library is missing.

Contents
--------
``reference``  float64 torch restatement of the reference algorithm:
               Psiformer forward (psiformer.py / blocks.py), local energy via a
               full autograd Hessian exactly as ``jax.hessian`` is used in
               hamiltonian.py:96-170, potential, MCMC proposal/accept with
               injected noise (mcmc.py), loss statistics (loss.py:30-92).
``channels``   an independent second restatement of the local energy by
               forward-mode (2N+5)-channel propagation — the algorithm the HIP
               kernels implement — used to debug the kernels layer by layer.
``philox``     numpy Philox4x32-10 + Box-Muller, bit-exact mirror of the
               device RNG used by the MCMC kernel.

Parity pinning: the reference (JAX/Flax, Python >= 3.11) cannot be imported in
this container (no jax/flax; Python 3.10 cannot parse hamiltonian.py:146).  The
oracle is pinned by the reference's own analytic known-answer tests
(tests/hamiltonian_test.py:42-76: free electrons KE=3, L^2=0; LLL Slater
determinants KE=N/2, L^2 in {2,0,0}) restated in ``tests/test_oracle_kat.py``,
by engineered-Psiformer known answers, by finite differences, and by agreement
of the two independent restatements.  The Psiformer forward values themselves
are not pinned by any reference fixture (none exists): "parity unpinned" for
raw log-psi values, see DESIGN.md.
"""
