"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the OneTrans training step.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product path (``recommend_amd``) never imports it and has no CPU fallback.

Parity status: the reference (TensorFlow 2.12, ``requirements.txt:1``) is not
installed here and cannot be installed offline, and the reference ships no tests,
golden vectors or fixtures for this path.  The oracle is
therefore **parity unpinned by the reference's own numerics**; it is pinned by
(i) hand-derived known-answer tests (tests/test_oracle.py), (ii) two
independent restatements (torch per-token ``literal`` vs numpy fp64
``onetrans_np``) that agree to 1e-12, and (iii) committed golden fixtures
generated from them (tests/golden/make_golden.py).  The reference's TensorFlow-free
code (config presets, PyramidScheduler, FeatureProcessor, SequenceProcessor) IS run
in the build container to produce fixtures (tests/golden/make_ref_fixtures.py,
checked by tests/test_reference_fixtures.py): those parts are pinned.
"""
