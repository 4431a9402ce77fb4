"""Diagnostic: vector-memory waits that stall right behind their own loads.

For every kernel of the built libdmdqn_hip.so (tools/disasm.py output), lists
each `s_waitcnt vmcnt(N)` that comes within WINDOW instructions of a
global/buffer load and waits for it (N smaller than the number of loads issued
since), with the instructions between.  The usual cause on this code base is
the wait-count insertion being conservative at a control-flow merge (a load or
a default value under a branch), which turns a look-ahead load into a
synchronous one ("conservative waits").
usage: python tools/waitcnt_audit.py [isa_dir] [kernel-substring] [window]"""
import glob
import re
import sys

isa = sys.argv[1] if len(sys.argv) > 1 else "/tmp/dmdqn_isa"
filt = sys.argv[2] if len(sys.argv) > 2 else ""
WINDOW = int(sys.argv[3]) if len(sys.argv) > 3 else 40

LOAD = re.compile(r"^(global_load|buffer_load|global_atomic\S*_rtn)")
for path in sorted(glob.glob(f"{isa}/*.s")):
    name, body = None, []
    kernels = []
    for line in open(path):
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            if name:
                kernels.append((name, body))
            name, body = m.group(1), []
            continue
        b = line.strip().split("//")[0].strip()
        if b:
            body.append(b)
    if name:
        kernels.append((name, body))
    for name, body in kernels:
        if filt not in name:
            continue
        hits = []
        for k, b in enumerate(body):
            m = re.match(r"s_waitcnt.*vmcnt\((\d+)\)", b)
            if not m:
                continue
            n = int(m.group(1))
            loads = [j for j in range(max(0, k - WINDOW), k) if LOAD.match(body[j])]
            if len(loads) > n:  # waits for at least one load issued in the window
                hits.append((k, n, len(loads), k - loads[len(loads) - n - 1]))
        if hits:
            print(f"{name[:90]}")
            for k, n, nl, dist in hits:
                print(f"   @{k}: vmcnt({n}) with {nl} loads in the last {WINDOW}; waits for one issued {dist} instr. before")
