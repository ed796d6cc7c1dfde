"""Step spread of schedule/launch variants (tools/variance_probe.py per variant, env settings per
variant, interleaved twice).  usage: python tools/variance_ab.py <calls> <variant> ...  where a
variant is "base" or "base@VAR=value[@VAR=value...]" (lib/abl/libykgpu_<name>.so for other names)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
calls = sys.argv[1]
for rnd in range(2):
    for name in sys.argv[2:]:
        lname, *envspecs = name.split("@")
        lib = os.path.join(ROOT, "uecraytracing_amd/lib/libykgpu.so") if lname == "base" else \
            os.path.join(ROOT, f"uecraytracing_amd/lib/abl/libykgpu_{lname}.so")
        env = dict(os.environ, YKGPU_LIB_OVERRIDE=lib)
        for envspec in envspecs:
            k, _, v = envspec.partition("=")
            env[k] = v
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools/variance_probe.py"), calls], env=env,
                             capture_output=True, text=True)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(rnd, name, out.stderr[-400:], flush=True)
            continue
        r = json.loads(line[-1])
        print(rnd, name, json.dumps({k: r[k] for k in ("ms_min", "ms_mean", "ms_max", "max_over_min")}), flush=True)
