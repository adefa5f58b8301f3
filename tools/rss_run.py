"""Run a command as a child process and report the peak resident set of its largest
descendant (resource.RUSAGE_CHILDREN ru_maxrss): the per-rank host memory of a bench run."""
import json
import resource
import subprocess
import sys
import time

t0 = time.time()
rc = subprocess.run(sys.argv[1:]).returncode
ru = resource.getrusage(resource.RUSAGE_CHILDREN)
print(json.dumps({"rc": rc, "max_rss_gib": ru.ru_maxrss / 2**20, "wall_s": time.time() - t0}), file=sys.stderr)
sys.exit(rc)
