"""Parity oracle for the SP-NeRF render path — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Nothing in sp-nerf_amd/ imports it: the product path runs on the HIP library or fails.
"""
