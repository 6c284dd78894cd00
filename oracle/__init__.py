"""CPU oracle for the DARE + QNN-alpha training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is imported by the product
package (``toss-next-ctr-prediction_amd/tossctr``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and
only as the checker / the timed CPU baseline -- never as the thing measured on
the GPU.

Parity status: PINNED.  ``tests/golden/*.npz`` were produced by
``tests/golden/gen_golden.py``, which imports the reference model code
(``/root/reference/src/models/*``, ``src/utils/{ema,sched}``) in the build
container and runs it on CPU; ``tests/test_oracle_golden.py`` checks this
restatement against those vectors.
"""
