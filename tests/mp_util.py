"""Collect results from spawned test workers without hanging: a worker that dies (exception, fault) ends the
wait at once instead of after the queue timeout."""
import queue
import time


def collect(procs, qret, n, timeout=300):
    out, t0 = [], time.time()
    while len(out) < n:
        try:
            out.append(qret.get(timeout=2))
            continue
        except queue.Empty:
            pass
        dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
        if dead:
            for p in procs:
                if p.is_alive():
                    p.terminate()
            raise RuntimeError(f"worker exited with {dead}")
        if time.time() - t0 > timeout:
            for p in procs:
                if p.is_alive():
                    p.terminate()
            raise TimeoutError(f"{len(out)}/{n} results after {timeout}s")
    return out
