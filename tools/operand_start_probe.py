"""Where an operand process's start-up goes (bench --mode process breakdown).

Every operand container is ``python -m amdgpu_operator <operand>``; its
``started_s`` in the bench's per-operand breakdown is interpreter start +
imports.  This probe splits that on the machine it runs on: bare interpreter
(with and without site), each operand's import set, the same with N processes
starting at once (a pod storm), and the top cumulative imports (-X importtime).
Prints one JSON object.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IMPORT_SETS = {
    "cli": "import amdgpu_operator.cli.main, amdgpu_operator.cli.operands",
    "validate": "import amdgpu_operator.cli.operands, amdgpu_operator.validator.validate, amdgpu_operator.kube.client",
    "device-plugin": "import amdgpu_operator.cli.operands, amdgpu_operator.deviceplugin.server",
    "driver": "import amdgpu_operator.cli.operands, amdgpu_operator.driver.manager",
    "toolkit": "import amdgpu_operator.cli.operands, amdgpu_operator.toolkit.install",
    "exporter": "import amdgpu_operator.cli.operands, amdgpu_operator.exporter.metrics",
}


def wall(argv, n=1, reps=5) -> float:
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        ps = [subprocess.Popen(argv, cwd=ROOT) for _ in range(n)]
        for p in ps:
            p.wait()
        best = min(best, time.perf_counter() - t)
    return round(best, 4)


def top_imports(code: str, k: int = 12) -> list:
    p = subprocess.run([sys.executable, "-X", "importtime", "-c", code], cwd=ROOT, capture_output=True, text=True)
    rows = []
    for line in p.stderr.splitlines():  # "import time:  self_us | cumulative_us | module"
        if not line.startswith("import time:") or "cumulative" in line:
            continue
        self_us, cum_us, name = (x.strip() for x in line[len("import time:"):].split("|"))
        rows.append((int(cum_us), int(self_us), name))
    rows.sort(reverse=True)
    return [{"module": n, "cumulative_ms": round(c / 1000, 2), "self_ms": round(s / 1000, 2)} for c, s, n in rows[:k]]


def main() -> None:
    py = sys.executable
    out = {"python": sys.version.split()[0], "cpus": os.cpu_count(),
           "bare_s": wall([py, "-c", "pass"]), "no_site_s": wall([py, "-S", "-c", "pass"]),
           "imports_s": {k: wall([py, "-c", v]) for k, v in IMPORT_SETS.items()},
           "concurrent_validate_s": {n: wall([py, "-c", IMPORT_SETS["validate"]], n=n, reps=3) for n in (1, 4, 8)},
           "top_imports_device_plugin": top_imports(IMPORT_SETS["device-plugin"])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
