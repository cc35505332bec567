"""CPU oracle for the SRF hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from this package, and only as the checker (or as the
timed CPU baseline).  The product path (``srf_amd``) never imports it.

Parity status: **unpinned against TensorFlow**.  The reference hot path
(``tfsr/model/sequence_router_naive.py``) imports TensorFlow at module level and
TensorFlow is not installed in this image (an ordinary ``ModuleNotFoundError``,
not a permission denial), and the reference ships no tests, golden vectors or
fixtures for this path.  The restatement is therefore
checked by (a) two independent implementations that must agree (the numpy
float64 ``srf_oracle`` and the torch ``naive_mirror`` op-for-op mirror), (b)
finite differences for gradients, (c) ``torch.nn.functional.ctc_loss`` for CTC.
The flag surface (``ParseOption``) *is* pinned against the reference itself,
whose ``tfsr/helper/common_helper.py`` is TF-free and was imported here to
produce ``tests/golden/flags_*.json`` (see ``oracle/gen_golden.py``).
"""
