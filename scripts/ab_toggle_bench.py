"""A/B helper: one bench.py workload with a module attribute set (e.g. gmp_amd.ops
EGNN_NODE_BWD_FUSED 0); prints the workload's edges/s and ms per step.
usage: ab_toggle_bench.py <workload> <module> <attr> <0|1> [steps]"""
import json
import subprocess
import sys

if __name__ == "__main__":
    wl, mod, attr, val = sys.argv[1:5]
    steps = sys.argv[5] if len(sys.argv) > 5 else "20"
    code = ("import sys, runpy, importlib; sys.path.insert(0, 'geometric-message-passing_amd'); "
            f"sys.argv = ['bench.py', '--workload', '{wl}', '--steps', '{steps}', '--warmup', '3', "
            "'--no-cpu-baseline', '--no-f32-exact', '--no-forward']; "
            f"setattr(importlib.import_module('{mod}'), '{attr}', bool({val})); "
            "runpy.run_path('bench.py', run_name='__main__')")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    o = d if wl == "egnn" else d.get(wl, d)
    print(f"{wl} {attr}={val}: {o['value'] / 1e6:.2f} M {o['ms_per_step']:.3f} ms")
