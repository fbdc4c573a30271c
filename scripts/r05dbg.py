"""One float and one 16-bit WINSORIZED stack per column capacity, each in
its own child process (a failing launch aborts only its child); prints which
capacity fails.  Diagnostic for the r05b abort."""
import subprocess
import sys

CODE = r'''
import sys, numpy as np
sys.path.insert(0, ".")
from siril_amd import stacking as S
n, u16 = int(sys.argv[1]), int(sys.argv[2])
rng = np.random.default_rng(n)
fr = (0.05 + 0.005 * rng.standard_normal((n, 4, 64))).astype(np.float32)
if u16:
    fr = np.round(fr * 30000).astype(np.uint16)
c = S.Context(0)
r = c.stack(fr, S.StackingArgs(S.Rejection.WINSORIZED, (3.0, 3.0)))
print("ok", n, u16, float(np.asarray(r.result).astype(np.float64).mean()), flush=True)
'''
for n in (100, 200, 400, 700, 1000, 30):
    for u16 in (0, 1):
        p = subprocess.run([sys.executable, "-c", CODE, str(n), str(u16)], capture_output=True, text=True, timeout=120)
        print(n, u16, "rc", p.returncode, p.stdout.strip()[-200:], flush=True)
        if p.returncode:
            print(p.stderr[-3000:], flush=True)
