"""Run several entry scripts in ONE torchrun job (one process per rank, one process
group): each script runs in-process as __main__ with its own argv, and the process group
is torn down once at the end (runtime.shutdown is a no-op in between). Saves the ~4 s
process + torch start-up per script of the one-GPU multi-rank rehearsal.

argv[1]: JSON list of [script path, [args...]]. Each script's output is framed by
==BEGIN i== / ==END i== lines (rank 0 prints the algorithm lines)."""
import json
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from dalgo.parallel import runtime  # noqa: E402


def main():
    jobs = json.loads(sys.argv[1])
    lead = os.environ.get("RANK", "0") == "0"      # rank 0 prints the algorithm lines
    real_shutdown = runtime.shutdown
    runtime.shutdown = lambda: None
    try:
        for i, (path, args) in enumerate(jobs):
            if lead:
                print(f"==BEGIN {i}==", flush=True)
            sys.argv = [path] + list(args)
            try:
                runpy.run_path(path, run_name="__main__")
            except SystemExit as e:
                if e.code not in (None, 0):
                    raise
            if lead:
                print(f"==END {i}==", flush=True)
    finally:
        runtime.shutdown = real_shutdown
    runtime.shutdown()


if __name__ == "__main__":
    main()
