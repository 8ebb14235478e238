"""Sanitized CPU builds (race detection / sanitizers): the C oracle (oracle/covis_oracle.c) and the host
session generator (csrc/synth.cpp) built with -fsanitize=address,undefined (`make -C oracle asan`,
`make -C otto-recommender_amd/csrc asan`) and run in a child process with libasan preloaded, on the Appendix-A
known-answer test, the 1k golden, a 3-file slice (the per-file count and the OpenMP files digest) and the generator's
sessions, item ranks and embeddings. Any ASan / UBSan report aborts the child (-fno-sanitize-recover); its results
must equal the ordinary builds'. No GPU is involved."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_ASAN = os.path.join(ROOT, "oracle", "_build", "libcovis_oracle_asan.so")
SYNTH_ASAN = os.path.join(ROOT, "otto-recommender_amd", "csrc", "build", "libottosynth_asan.so")

CHILD = r"""
import json, sys
import numpy as np
sys.path[:0] = [{root!r}, {oracle!r}]
import covis
import otto_recommender_amd.synth as synth
g = json.load(open({kat!r}))
a = np.array(g["events"])
ev = synth.events_from_columns(a[:, 0], a[:, 1], a[:, 2], a[:, 3])
kat = covis.count_co_events_file(ev.session_offsets, ev.aid, ev.ts, ev.type)
out = {{"kat": {{k: [[int(x), int(y), int(c)] for x, y, c in zip(*v)] for k, v in kat.items()}}}}
ev = synth.generate(1000)
t = covis.count_co_events_file(ev.session_offsets, ev.aid, ev.ts, ev.type)
out["g1k"] = covis.canonical_digest({{k: v for k, v in t.items()}})
ev = synth.generate(3000, first_session=777_777)
fb = np.array([0, 700, 2100, 3000], np.int64)
out["files"] = [covis.canonical_digest(p) for p in covis.count_co_events_files(ev.session_offsets, ev.aid, ev.ts,
                                                                              ev.type, fb)]
out["files_digest"] = covis.files_digest(ev.session_offsets, ev.aid, ev.ts, ev.type, fb, threads=4)
out["synth"] = [int(ev.session_offsets[-1]), int(np.sum(ev.aid.astype(np.int64))), int(np.sum(ev.ts.astype(np.int64))),
                int(synth.item_rank(n_items=50_000)[:1000].astype(np.int64).sum()),
                float(synth.embeddings(2000, seed=3).astype(np.float64).sum())]
maps = open("/proc/self/maps").read()
loaded = [n for n in ("libasan", "libcovis_oracle_asan.so", "libottosynth_asan.so") if n in maps]
print("LOADED " + json.dumps(loaded))
print("RESULT " + json.dumps(out, sort_keys=True))
"""


def _run(env_extra):
    code = CHILD.format(root=ROOT, oracle=os.path.join(ROOT, "oracle"),
                        kat=os.path.join(ROOT, "tests", "golden", "kat_appendix_a.json"))
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    loaded = json.loads([x for x in r.stdout.splitlines() if x.startswith("LOADED ")][-1][len("LOADED "):])
    return json.loads(line[-1][len("RESULT "):]), r.stderr, loaded


def test_oracle_and_generator_under_asan_ubsan():
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(libasan):
        pytest.skip("gcc's libasan is not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "otto-recommender_amd", "csrc"), "asan"], check=True)
    plain, _, loaded = _run({})
    assert loaded == []
    san, err, loaded = _run({"LD_PRELOAD": libasan, "OTTO_ORACLE_SO": ORACLE_ASAN, "OTTOSYNTH_SO": SYNTH_ASAN,
                     "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
                     "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"})
    assert "runtime error" not in err and "AddressSanitizer" not in err, err[-4000:]
    assert loaded == ["libasan", "libcovis_oracle_asan.so", "libottosynth_asan.so"]  # the sanitized builds ran
    assert san == plain
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat_appendix_a.json")))["expected"]
    assert san["kat"] == kat
