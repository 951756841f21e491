"""Run a test body against the diagnostic build of the library (libfloam_amd_diag.so, FLOAM_AMD_LIB=diag).

The product library reads no A/B or test-hook environment variables (floam_amd/csrc/floam_common.hpp FLOAM_DIAG_ENV);
a test that needs a hook (a forced fallback, an injected fault or delay) runs its body in a spawned process that loads
the diagnostic build with the hook's variables set.  The body must be a module-level function; its return value comes
back through a queue (numpy arrays, tuples, dicts)."""
import multiprocessing as mp
import os
import traceback


def _child(q, fn, args):
    try:
        q.put(("ok", fn(*args)))
    except BaseException:   # noqa: BLE001 (reported to the parent)
        q.put(("error", traceback.format_exc()))


def run_diag(fn, *args, env=None, timeout=300):
    """fn(*args) in a fresh process on the diagnostic library with the variables `env` set; returns its result."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    full = {"FLOAM_AMD_LIB": "diag", **(env or {})}
    saved = {k: os.environ.get(k) for k in full}
    os.environ.update(full)   # (inherited by the spawned process from its start)
    try:
        p = ctx.Process(target=_child, args=(q, fn, args))
        p.start()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        status, val = q.get(timeout=timeout)
    finally:
        p.join(timeout=60)
    if status != "ok":
        raise AssertionError(f"diagnostic-build run failed:\n{val}")
    assert p.exitcode == 0, p.exitcode
    return val
