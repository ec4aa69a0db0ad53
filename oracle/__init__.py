"""ORACLE — test infrastructure only (see oracle/ref_cpu.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the timed CPU baseline; the product
path (pixel-nerf_amd/) never imports it.
"""
