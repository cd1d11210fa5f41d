"""Non-driver node of a multi-node engine: runs ranks [node_rank*g, (node_rank+1)*g)
of a TP x PP engine whose driver (node 0, the API server) lives in another pod.

This is the in-house replacement for the reference's KubeRay worker group (multi-pod
pipeline parallelism, ``values-01-minimal-example4.yaml:42-46``, ``old_README.md:
1564-1624``).  The ranks rendezvous with torch.distributed at ``--master-addr`` and
then execute the driver's broadcast step commands until it exits.

    python -m kubernetes_gpu_cluster_amd.entrypoints.worker_node MODEL \\
        --tensor-parallel-size 2 --pipeline-parallel-size 2 --nnodes 2 --node-rank 1 \\
        --master-addr leader-0.leader.default.svc --health-port 8000

``--node-rank`` defaults to ``$NODE_RANK``, else the pod ordinal
(``apps.kubernetes.io/pod-index`` via ``$POD_INDEX``, or the hostname suffix) plus
``--node-rank-offset``.  ``--health-port`` serves ``GET /health`` (200 while every local
rank is alive) for the pod's probes.
"""
from __future__ import annotations

import argparse
import http.server
import logging
import os
import re
import socket
import sys
import threading
import time

from ..engine.config import add_engine_args, config_from_args
from ..engine.worker import spawn_local_ranks

log = logging.getLogger("kgc.worker_node")


def _pod_ordinal() -> int | None:
    for k in ("POD_INDEX", "JOB_COMPLETION_INDEX"):
        v = os.environ.get(k)
        if v not in (None, ""):
            return int(v)
    m = re.search(r"-(\d+)$", socket.gethostname())
    return int(m.group(1)) if m else None


def _serve_health(port: int, procs) -> None:
    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            ok = self.path.startswith("/health") and all(p.is_alive() for p in procs)
            self.send_response(200 if ok else 503)
            self.end_headers()
            self.wfile.write(b"ok" if ok else b"rank down")

        def log_message(self, *a):
            pass
    srv = http.server.ThreadingHTTPServer(("0.0.0.0", port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()


def make_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="kgc multi-node engine worker")
    p.add_argument("model_tag", nargs="?", default=None)
    p.add_argument("--node-rank-offset", type=int, default=0,
                   help="added to the pod ordinal when --node-rank/$NODE_RANK are not given")
    p.add_argument("--health-port", type=int, default=0)
    add_engine_args(p)
    return p


def main(argv=None) -> int:
    p = make_parser()
    ns = p.parse_args(argv)
    ns.model = ns.model or ns.model_tag or "llama-3-8b"
    explicit = any(a == "--node-rank" or a.startswith("--node-rank=") for a in (argv or sys.argv[1:]))
    if not explicit:
        if os.environ.get("NODE_RANK"):
            ns.node_rank = int(os.environ["NODE_RANK"])
        else:
            o = _pod_ordinal()
            if o is None:
                p.error("cannot infer --node-rank (no $NODE_RANK, $POD_INDEX or ordinal hostname)")
            ns.node_rank = o + ns.node_rank_offset
    cfg = config_from_args(ns)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")
    if not 1 <= cfg.node_rank < cfg.nnodes:
        p.error(f"--node-rank {cfg.node_rank} must be in [1, {cfg.nnodes}) (node 0 is the driver)")
    g = cfg.ranks_per_node
    first = cfg.node_rank * g
    env = cfg.dist_env()
    for k in ("HSA_ENABLE_IPC_MODE_LEGACY", "KGC_DIST_BACKEND"):
        if k in os.environ:
            env[k] = os.environ[k]
    log.info("node %d/%d: ranks %d..%d -> %s:%s", cfg.node_rank, cfg.nnodes, first, first + g - 1,
             env["MASTER_ADDR"], env["MASTER_PORT"])
    procs = spawn_local_ranks(cfg, env, first, first + g, daemon=False)
    if ns.health_port:
        _serve_health(ns.health_port, procs)
    # exit when any rank exits: a failed rank must take the pod down (restart), and the
    # driver's shutdown (CMD_EXIT) ends every rank cleanly
    rc = 0
    while procs:
        for pr in list(procs):
            if not pr.is_alive():
                procs.remove(pr)
                if pr.exitcode:
                    rc = pr.exitcode
                    log.error("rank process %s exited with %s", pr.pid, pr.exitcode)
        if rc:
            for pr in procs:
                pr.terminate()
            break
        time.sleep(0.5)
    return rc


if __name__ == "__main__":
    sys.exit(main())
