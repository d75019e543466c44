#!/usr/bin/env python3
"""Check the two-pods-one-gpu Job: every pod passed vectorAdd on exactly one, distinct MI355X.

The reference verifies GPU isolation by eye — two pods print their GPU UUIDs and a human compares
them (reference README.md:301-387).  This turns that into a pass/fail check over the pods' logs
(cluster-config/apps/gpu-bench/job-two-pods-one-gpu.yaml prints kfd-probe's JSON, which carries
each visible agent's unique_id, then the vectorAdd protocol).

    scripts/check_isolation.py                 # reads logs with kubectl
    scripts/check_isolation.py pod1.log pod2.log
"""
import json
import subprocess
import sys
from typing import Dict, List, Tuple


def parse_pod_log(text: str) -> dict:
    probe = None
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{") and '"agents"' in line:
            try:
                probe = json.loads(line)
            except ValueError:
                pass
    lines = [ln.strip() for ln in text.splitlines() if ln.strip()]
    passed = "Test PASSED" in lines and "Done" in lines and "Test FAILED" not in lines
    uids = [a.get("unique_id") for a in (probe or {}).get("agents", [])]
    return {"passed": passed, "gpu_unique_ids": uids, "probe_ok": bool(probe and probe.get("ready"))}


def check(logs: Dict[str, str]) -> Tuple[bool, List[str]]:
    report, seen, ok = [], {}, True
    for pod, text in sorted(logs.items()):
        r = parse_pod_log(text)
        report.append(f"{pod}: passed={r['passed']} gpus={r['gpu_unique_ids']}")
        if not r["passed"] or len(r["gpu_unique_ids"]) != 1:
            ok = False
            report.append(f"  FAIL: {pod} must pass vectorAdd and see exactly one GPU")
            continue
        uid = r["gpu_unique_ids"][0]
        if uid in seen:
            ok = False
            report.append(f"  FAIL: {pod} shares GPU {uid} with {seen[uid]}")
        seen[uid] = pod
    if len(logs) < 2:
        ok = False
        report.append("FAIL: expected at least two pods")
    return ok, report


def kubectl_logs(namespace: str = "gpu-bench", job: str = "two-pods-one-gpu") -> Dict[str, str]:
    pods = subprocess.run(["kubectl", "-n", namespace, "get", "pods", "-l", f"job-name={job}", "-o",
                           "jsonpath={.items[*].metadata.name}"], capture_output=True, text=True,
                          check=True).stdout.split()
    return {p: subprocess.run(["kubectl", "-n", namespace, "logs", p], capture_output=True, text=True,
                              check=True).stdout for p in pods}


def main(argv) -> int:
    logs = {p: open(p).read() for p in argv} if argv else kubectl_logs()
    ok, report = check(logs)
    print("\n".join(report))
    print("ISOLATION OK" if ok else "ISOLATION FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
