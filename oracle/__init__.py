"""ORACLE -- TEST INFRASTRUCTURE ONLY.

A CPU restatement of the reference's sampling hot path (tommyod/probabilit @ 2025-09-19),
used as the checker by tests/, by __graft_entry__.smoke() and by bench.py's cpu_baseline
leg.  Nothing in probabilit_amd imports, links or executes anything under oracle/.

Modules
    streams   PCG64 / Latin hypercube / Sobol' restatements of the scipy 1.15.3 engines the
              reference calls at modeling.py:479-489 (pure Python / numpy, small n)
    ppf       the reference's inverse-CDF call (modeling.py:807) on scipy 1.15.3, the
              reference's own pinned L0 dependency, present in this image
    ic        numpy restatement of ImanConover.__call__ (correlation.py:368-425) with every
              intermediate exposed, including its own restatement of rankdata('average')
    pipeline  the BASELINE.json configurations end to end (LHS + ppf + IC; mutual fund)

Pinning: tests/test_oracle.py checks every function here against the golden vectors in
tests/golden/*.npz, which tests/golden/make_golden.py produced by running the reference
itself (stub-imported) in the build container.
"""
