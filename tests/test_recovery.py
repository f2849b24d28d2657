"""Elastic recovery of a model-parallel server: a TP=2 group on CPU (gloo)
under ``torchrun --max-restarts 1`` with an injected rank failure (NGA_FAULT) goes down and
comes back serving on the same port; a wedged rank is turned into a restart by the driver's
fail-fast watchdog."""
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _post(url, body, timeout=30):
    req = urllib.request.Request(url, data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.status, json.loads(r.read())


@pytest.mark.parametrize("fault", ["crash@rank1:step3", "hang@rank1:step3"])
def test_tp_group_restarts_after_rank_failure(fault, tmp_path):
    http, master = _free_port(), _free_port()
    env = dict(os.environ, NGA_FAULT=fault, OMP_NUM_THREADS="2", LOGLEVEL="WARNING",
               PYTHONPATH=os.getcwd())
    log = open(tmp_path / "tp.log", "w")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--max-restarts=1", "--monitor-interval=0.5", "--rdzv-backend=c10d",
           f"--rdzv-endpoint=127.0.0.1:{master}", "-m", "nv_genai_amd.serving.tp_server", "--llm", "llama-tiny",
           "--tp", "2", "--port", str(http), "--max-num-seqs", "4", "--max-model-len", "512",
           "--watchdog-s", "6"]
    proc = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    url = f"http://127.0.0.1:{http}/v1/completions"
    body = {"prompt": "recover me", "max_tokens": 8, "ignore_eos": True, "temperature": 0.0}
    failures, ok = 0, None
    try:
        deadline = time.time() + 240
        while time.time() < deadline:   # first incarnation up
            assert proc.poll() is None, open(tmp_path / "tp.log").read()[-3000:]
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{http}/v1/health/ready", timeout=5):
                    break
            except Exception:  # noqa: BLE001
                time.sleep(0.5)
        while time.time() < deadline and ok is None:
            assert proc.poll() is None, open(tmp_path / "tp.log").read()[-3000:]
            try:
                st, out = _post(url, body)
                if st == 200 and out["choices"][0]["finish_reason"] == "length":
                    if failures:
                        ok = out
                    else:       # served before the fault step: keep going until it fires
                        continue
            except Exception:   # noqa: BLE001 - connection refused / reset / 500 while down
                failures += 1
                time.sleep(0.5)
        assert ok is not None, open(tmp_path / "tp.log").read()[-3000:]
        assert failures >= 1 and ok["usage"]["completion_tokens"] == 8
    finally:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(timeout=20)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait()
