"""CPU oracle for the CiM hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package; the product (``cim_quantization_amd``) never does.
"""
