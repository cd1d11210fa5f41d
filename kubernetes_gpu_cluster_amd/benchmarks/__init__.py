"""Benchmark harness pieces shared by ``bench.py`` and ``bench/serve_bench.py``."""
