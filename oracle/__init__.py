"""CPU oracle for the ship-in-transit env step — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the reported CPU baseline.  The product
path (``sac_maritime_ast_amd``) never imports it and fails loudly without its HIP library.
"""
