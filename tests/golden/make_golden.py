"""Regenerate the golden fixtures in tests/golden/ (run in the build container).

Inputs are data the reference's own tests hold, read from /root/reference at
generation time only (the GPU box never reads it):
  * service/worker/archiver/testdata/archival_workflow_history_v1.json (112 events)
  * the hex-encoded JSON history of service/history/timerBuilder_test.go:218
Expected outputs are produced by the CPU restatement (oracle/), which is itself
pinned by tests/test_oracle_kat.py (the reference's known-answer tests); the Go
stateBuilder cannot run here (no Go toolchain), so these are oracle-generated
goldens, frozen so that any later change to the oracle or the engine is caught.
Also written: digests of small synthetic batches of every SURVEY §8(d) config.
"""
import hashlib
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
from cadence_amd import abi, engine  # noqa: E402
from cadence_amd.history import from_cadence_json  # noqa: E402

REF = "/root/reference"
SYNTH = [(cfg, 64, 0x5EED0000 + cfg, 0.0) for cfg in (1, 2, 3, 4, 5)] + [(0, 96, 0x5EED00F0, 0.25),
                                                                          (3, 96, 0x5EED00F3, 0.25)]


def load_inputs():
    arch = json.load(open(f"{REF}/service/worker/archiver/testdata/archival_workflow_history_v1.json"))
    src = open(f"{REF}/service/history/timerBuilder_test.go").read()
    tb = json.loads(bytes.fromhex(re.search(r'historyString := "([0-9a-f]+)"', src).group(1)))
    return {"archival_workflow_history_v1": arch, "timer_builder_history": tb}


def replay_json(events, batching):
    b = from_cadence_json(events, workflow_id="golden-wid", run_id="golden-rid", request_id="golden-req",
                          builder=abi.BUILDER_NDC, failover_version=abi.EMPTY_VERSION, batching=batching)
    return b, oracle.replay(b)


def digest(batch, out):
    return engine.state_digest(batch, out)


def main():
    for name, events in load_inputs().items():
        json.dump(events, open(os.path.join(HERE, f"{name}.input.json"), "w"), indent=0)
        exp = {}
        for batching in ("single", "each"):
            b, out = replay_json(events, batching)
            exp[batching] = engine.export_state(b, out, 0)
        json.dump(exp, open(os.path.join(HERE, f"{name}.expected.json"), "w"), indent=1, sort_keys=True)
    syn = {}
    for cfg, n, seed, er in SYNTH:
        b = engine.synth_batch(cfg, n, seed, error_rate=er)
        out = oracle.replay(b)
        syn[f"{cfg}:{n}:{seed}:{er}"] = {"digest": digest(b, out), "status": engine.status_histogram(out),
                                         "first": engine.export_state(b, out, 0)}
    json.dump(syn, open(os.path.join(HERE, "synthetic.expected.json"), "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
