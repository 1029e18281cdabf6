"""Where a one-shot `ciruela-index sync` spends its time (config 1's
cli_seconds): wall time of the process with no arguments (dynamic loading
only), of a bare HIP start-up (build/hip_start_probe), and of the sync of a
100-file / 10 MiB tree with CIR_TRACE=1 (HIP runtime start, cir_init, the
scan, cir_destroy as the CLI reports them).

    python tools/cli_startup.py [--runs 5] [--ab-teardown]

--ab-teardown: only the sync, alternating the default exit (no cir_destroy)
with CIR_CLI_TEARDOWN=1, without CIR_TRACE; prints each run and the medians.
"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def timed(cmd, env=None):
    t0 = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, text=True, env=env)
    return time.perf_counter() - t0, p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--ab-teardown", action="store_true")
    ap.add_argument("--ab-env", default="CIR_CLI_TEARDOWN",
                    help="the variable --ab-teardown alternates between 0 and 1")
    args = ap.parse_args()
    cli = os.path.join(ROOT, "bin", "ciruela-index")
    probe = os.path.join(ROOT, "build", "hip_start_probe")
    with tempfile.TemporaryDirectory() as tmp:
        tree = os.path.join(tmp, "tree")
        for i in range(100):
            d = os.path.join(tree, "d%d" % (i % 10))
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, "f%03d" % i), "wb") as f:
                f.write(os.urandom(100 << 10) if i < 99 else os.urandom((10 << 20) - 99 * (100 << 10)))
        if args.ab_teardown:
            runs = {"exit": [], "teardown": []}
            for r in range(args.runs):
                for mode in ("exit", "teardown"):
                    env = dict(os.environ, **{args.ab_env: "1" if mode == "teardown" else "0"})
                    s, p = timed([cli, "sync", "--append", tree + ":/x"], env)
                    if p.returncode:
                        print(p.stderr)
                        sys.exit(p.returncode)
                    runs[mode].append(s * 1e3)
                    print("%s %.1f ms | %s" % (mode, s * 1e3, p.stdout.split()[0]), flush=True)
            for mode, v in runs.items():
                print("median %s=%s %.1f ms over %d runs" % (args.ab_env, "1" if mode == "teardown" else "0",
                                                         sorted(v)[len(v) // 2], len(v)))
            return
        for r in range(args.runs):
            s, _ = timed([cli])
            print("no-args (load only) %.1f ms" % (s * 1e3), flush=True)
        for r in range(args.runs):
            s, p = timed([probe])
            print("hip_start_probe %.1f ms | %s" % (s * 1e3, p.stdout.strip().replace("\n", "; ")),
                  flush=True)
        env = dict(os.environ, CIR_TRACE="1")
        for r in range(args.runs):
            s, p = timed([cli, "sync", "--append", tree + ":/x"], env)
            if p.returncode:
                print(p.stderr)
                sys.exit(p.returncode)
            lines = [ln for ln in p.stderr.splitlines()
                     if ln.startswith(("ciruela-index:", "Indexed", "cir_init dev"))]
            print("sync %.1f ms | %s" % (s * 1e3, "; ".join(lines)), flush=True)


if __name__ == "__main__":
    main()
