"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference (k0r1g/two-towers) hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker / the timed CPU baseline.  The product (twotower_amd) never imports it
and has no CPU fallback.

Pinning: every function is checked in tests/test_oracle_golden.py against golden vectors that
tests/golden/make_golden.py captured by running the reference's own modules
(/root/reference/twotower/{embeddings,encoders,losses}.py and torch.optim.AdamW) in the build
container.  The reference ships no tests or fixtures for this path, so those
captured vectors are the pin.
"""
