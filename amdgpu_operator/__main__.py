import os
import sys
import time

if os.environ.get("AMDGPU_STARTUP_TRACE"):  # the interpreter is up (cli/main.py marks the later phases)
    with open(os.environ["AMDGPU_STARTUP_TRACE"], "a") as _f:
        _f.write(f"interp {time.time():.4f}\n")

if sys.flags.no_site:
    # Operand containers start as `python3 -S -m amdgpu_operator` (images:
    # tools/image_manifest.py; the simulated kubelet: testing/simcluster.py):
    # `site` and the .pth files it executes cost a fresh interpreter ~13 ms on
    # the MI355X box (~35 ms here), on every operand's start-up path.  The
    # images carry their dependencies on PYTHONPATH; elsewhere the
    # interpreter's package directories are appended, without .pth processing.
    _v = f"python{sys.version_info[0]}.{sys.version_info[1]}"
    for _d in (os.path.join(sys.prefix, "local", "lib", _v, "dist-packages"),
               os.path.join(sys.prefix, "lib", "python3", "dist-packages"),
               os.path.join(sys.prefix, "lib", _v, "dist-packages"),
               os.path.join(sys.prefix, "lib", _v, "site-packages")):
        if os.path.isdir(_d) and _d not in sys.path:
            sys.path.append(_d)

from .cli.main import main

sys.exit(main())
