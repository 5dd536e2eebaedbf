"""bench.py's GVP workload with K17 switched by GMP_AB_FF (A/B helper; prints edges/s, ms)."""
import json
import os
import subprocess
import sys



if __name__ == "__main__":
    code = ("import sys, runpy; sys.path.insert(0, 'geometric-message-passing_amd'); sys.argv = ['bench.py', '--workload', 'gvp', '--steps', '20', "
            "'--warmup', '3', '--no-cpu-baseline', '--no-f32-exact', '--no-forward']; "
            "import gmp_amd.gvp as g; g.GVP_FF_FUSED = " +
            ("True" if os.environ.get("GMP_AB_FF", "1") == "1" else "False") +
            "; runpy.run_path('bench.py', run_name='__main__')")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    o = d.get("gvp", d)
    print(round(o["value"] / 1e6, 2), "M", round(o["ms_per_step"], 3), "ms")
