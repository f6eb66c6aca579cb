"""C5 in the reference's process shape: the seeder and the leecher as two OS
processes (two test_client runs, cpp/test_client/src/test_client.cpp:27-77;
SURVEY.md §3.3 "This is the process boundary").

`lbf_loopback --role seeder` writes the flood file, listens on 127.0.0.1 and
publishes its port in a file; `lbf_loopback --role leecher --port P` loads the
flood file and downloads.  Each is a fresh child process with its own HIP
runtime, GPU contexts, arenas and registrations.  run_pair() starts both with
the same options and merges their two JSON lines into the one-process line's
shape (the leecher's line, with the seeder's own counters filled in).

    python -m tests.c5_pair --size 17179869184 --synthetic ...   # one merged line
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOOPBACK = os.path.join(ROOT, "bitflood_amd", "lib", "lbf_loopback")


def _last_json(text):
    lines = [ln for ln in text.strip().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def run_pair(args, directory, timeout=600, start_timeout=300):
    """args: lbf_loopback options without --role/--dir/--port.  Returns
    (merged, seeder_line, leecher_line); raises AssertionError with both
    processes' stderr when either fails."""
    os.makedirs(directory, exist_ok=True)
    port_file = os.path.join(directory, "seeder.port")
    common = [LOOPBACK] + list(args) + ["--dir", directory]
    t0 = time.monotonic()
    seeder = subprocess.Popen(common + ["--role", "seeder", "--port-file", port_file],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    leecher = None
    try:
        while not os.path.exists(port_file):
            if seeder.poll() is not None:
                out, err = seeder.communicate()
                raise AssertionError(f"seeder exited {seeder.returncode} before listening:\n{err}{out}")
            if time.monotonic() - t0 > start_timeout:
                raise AssertionError(f"seeder did not publish its port within {start_timeout} s")
            time.sleep(0.02)
        with open(port_file) as f:
            port = int(f.read().strip())
        left = max(10.0, timeout - (time.monotonic() - t0))
        leecher = subprocess.run(common + ["--role", "leecher", "--port", str(port)],
                                 capture_output=True, text=True, timeout=left)
        s_out, s_err = seeder.communicate(timeout=120)
    finally:
        if seeder.poll() is None:
            seeder.kill()
            seeder.wait()
    assert leecher.returncode == 0 and seeder.returncode == 0, (
        f"leecher exit {leecher.returncode}, seeder exit {seeder.returncode}\n"
        f"leecher stderr:\n{leecher.stderr}\nseeder stderr:\n{s_err}\n{leecher.stdout}{s_out}")
    sl, ll = _last_json(s_out), _last_json(leecher.stdout)
    assert sl and sl["role"] == "seeder", s_out
    assert ll and ll["role"] == "leecher", leecher.stdout
    merged = dict(ll)
    merged["seeder"] = sl["seeder"]
    merged["corrupted_sent"] = sl["corrupted_sent"]
    merged["encode_flood_s"] = sl["encode_flood_s"]
    merged["process_shape"] = "two processes"
    merged["pids"] = {"seeder": sl["pid"], "leecher": ll["pid"]}
    return merged, sl, ll


def main(argv):
    with tempfile.TemporaryDirectory(prefix="c5_pair_", dir=os.environ.get("TMPDIR")) as d:
        merged, _, _ = run_pair(argv, os.path.join(d, "c5"), timeout=1800)
    print(json.dumps(merged))
    return 0 if merged["resume_verify_complete"] and merged["files_identical"] else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
