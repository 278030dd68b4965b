"""Build A/B variant libraries of librfrt.so into tools/_var/lib_<name>.so, one per NAME=FLAGS
argument (FLAGS: space-separated -D options added to the library's own flags), e.g.

    python tools/build_variants.py ldsstack16="-DRT_BVH_LDS_STACK=16" rowx2="-DRT_ROW_X2=1"

Each variant gets its own object directory (tools/_var/obj_<name>); tools/gpu.sh's covvar /
tracevar / k2var tasks then run every tools/_var/lib_*.so against librfrt.so."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
VAR = os.path.join(HERE, "_var")


def main(args):
    os.makedirs(VAR, exist_ok=True)
    for a in args:
        name, _, flags = a.partition("=")
        env = dict(os.environ, RFRT_BUILD_DIR=os.path.join(VAR, f"obj_{name}"),
                   RFRT_LIB_OUT=os.path.join(VAR, f"lib_{name}.so"), RFRT_EXTRA_CFLAGS=flags)
        r = subprocess.run([sys.executable, "-m", "rf_ray_tracing_warp_amd.build"], env=env,
                           cwd=os.path.dirname(HERE), capture_output=True, text=True)
        if r.returncode:
            sys.exit(f"{name}: build failed\n{r.stderr[-3000:]}")
        print(f"{name}: {env['RFRT_LIB_OUT']} ({flags})")


if __name__ == "__main__":
    main(sys.argv[1:])
