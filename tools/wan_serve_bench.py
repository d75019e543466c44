#!/usr/bin/env python3
"""The Wan2.1 ComfyUI-compatible server on one MI355X with full-size random-init models under the
reference's file names: start-up warm-up (model load, MIOpen compile + solver search, HIP-graph
capture), then the reference client's job (512x320, 16 frames, 25 uni_pc steps, CFG 6, animated
WEBP) submitted through the HTTP API and timed from POST /prompt to the file on disk."""
import json
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fastapi.testclient import TestClient  # noqa: E402

from k8s_nvidia_gpus_amd.models.comfy_client import ComfyClient, WanJob, build_wan_graph  # noqa: E402
from k8s_nvidia_gpus_amd.models.wan.server import create_app, synthetic_store  # noqa: E402


def heartbeat():
    t0 = time.time()

    def run():
        while True:
            time.sleep(30)
            print(f"[wan_serve_bench] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def main():
    heartbeat()
    out = tempfile.mkdtemp()
    t0 = time.time()
    app = create_app(synthetic_store("cuda"), out, ffmpeg="", warmup=(512, 320, 16))
    res = {}
    with TestClient(app) as c:
        assert app.state.ready.wait(900), "warm-up did not finish"
        res["ready_s"] = round(time.time() - t0, 1)
        lat = []
        for seed in range(3):
            job = WanJob(prompt=f"a panda riding a motorbike, take {seed}", seed=seed, formats=("webp",))
            t1 = time.perf_counter()
            pid = c.post("/prompt", json={"prompt": build_wan_graph(job)}).json()["prompt_id"]
            assert app.state.queue.wait_idle(600)
            h = c.get(f"/history/{pid}").json()[pid]
            assert h["status"]["status_str"] == "success", h["status"]
            f = ComfyClient.output_files(h)[0]
            size = len(c.get("/view", params=f).content)
            lat.append(round(time.perf_counter() - t1, 3))
            res.setdefault("files", []).append({"name": f["filename"], "bytes": size,
                                                "exec_s": h["meta"]["execution_s"]})
        res["request_s"] = lat
        # burst: 4 prompts queued at once — sampling of prompt i+1 overlaps the WEBP encode of i
        t1 = time.perf_counter()
        pids = [c.post("/prompt", json={"prompt": build_wan_graph(
            WanJob(prompt=f"burst {i}", seed=10 + i, formats=("webp",)))}).json()["prompt_id"]
            for i in range(4)]
        assert app.state.queue.wait_idle(900)
        assert all(c.get(f"/history/{p}").json()[p]["status"]["status_str"] == "success" for p in pids)
        res["burst4_s"] = round(time.perf_counter() - t1, 3)
    res["job"] = "512x320, 16 frames (13 decoded), 25 uni_pc/simple steps, CFG 6, animated WEBP"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
