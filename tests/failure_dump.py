"""Keep the data of a failing comparison: a test that compares two
sides on a state it generated itself (a trained snapshot, a drawn batch) wraps its assertions in
`dump_on_failure(...)`; when one of them fails, the arrays and the JSON-able records it was given
are written under a directory (default gpurun_out/failures/<name>/, which gpurun returns) and the
assertion is re-raised, so the next failure is diagnosed from its own data instead of a pattern.

Size: gpurun merges at most 64 MiB of gpurun_out/ back, so callers pass what re-running the
comparison needs (parameters, grid, batch, noise, the decisions both sides took) and leave out what
can be regenerated or is only derived."""
import contextlib
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_DIR = os.environ.get("NCN_FAILURE_DUMP_DIR") or os.path.join(ROOT, "gpurun_out", "failures")


def _jsonable(x):
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, np.ndarray):
        return x.tolist() if x.size <= 4096 else f"<array {x.dtype} {x.shape}>"
    if isinstance(x, (np.floating, np.integer, np.bool_)):
        return x.item()
    if hasattr(x, "detach"):  # a torch tensor
        return _jsonable(x.detach().cpu().numpy())
    return x


def write_dump(name, arrays, records, base=None):
    """arrays: {key: array-like} -> <dir>/arrays.npz (compressed); records: JSON-able -> record.json."""
    d = os.path.join(base or DEFAULT_DIR, name)
    os.makedirs(d, exist_ok=True)
    arr = {}
    for k, v in arrays.items():
        if v is None:
            continue
        if hasattr(v, "detach"):
            v = v.detach().cpu().numpy()
        arr[k] = np.asarray(v)
    np.savez_compressed(os.path.join(d, "arrays.npz"), **arr)
    with open(os.path.join(d, "record.json"), "w") as f:
        json.dump(_jsonable(records), f, indent=1, default=str)
    return d


@contextlib.contextmanager
def dump_on_failure(name, arrays, records, base=None):
    """Run the block; on an AssertionError write the dump (arrays / records may be callables that
    build them lazily) and re-raise with the dump's path appended."""
    try:
        yield
    except AssertionError as e:
        a = arrays() if callable(arrays) else arrays
        r = records() if callable(records) else records
        path = write_dump(name, a, dict(r, failure=str(e)[:20000]), base=base)
        raise AssertionError(f"{e}\n[failure data written to {path}]") from e
