#!/usr/bin/env python3
"""Generate a link-time stub of the HIP runtime whose SONAME is plain `libamdhip64.so`.

liborbamd.so is linked against this stub so its DT_NEEDED entry is `libamdhip64.so`:
inside a Python process that has imported torch, the loader then binds liborbamd.so to
the HIP runtime torch already loaded (one runtime per process -- two runtimes cannot share
devices or pointers); elsewhere RUNPATH resolves it to /opt/rocm/lib/libamdhip64.so.
The stub is never loaded at run time."""
import subprocess
import sys

objs = sys.argv[2:]
out = sys.argv[1]
syms = set()
for o in objs:
    for line in subprocess.check_output(["nm", "-u", o], text=True).splitlines():
        name = line.split()[-1]
        if name.startswith(("hip", "__hip")):
            syms.add(name)
src = "".join("void %s(void) {}\n" % s for s in sorted(syms))
open(out, "w").write(src)
