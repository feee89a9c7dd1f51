"""Pool ingest: the reference's text format -> pinned host memory -> HBM.

Reference: final_thesis/uncertainty_sampling.py:37-42 and
density_weighting.py:45-53,59-65 read whitespace rows (features, label last)
with ``sc.textFile``, map the label ``0 if int(_[-1]) == -1 else 1`` and the
features ``np.array(_[:-1]).astype(float)``, and keep ``take(n_samples)``.

Here the file is memory-mapped and parsed by the native multi-threaded parser
(libdal ``dal_parse_labeled_text``, C ABI in include/dal.h) straight into
page-locked host buffers, in row chunks; each chunk's host->device copy is
issued asynchronously on a side stream while the next chunk is parsed, so the
PCIe upload overlaps the parse.  The pool lands in HBM as fp32 row-major
[N, D] (the layout every kernel reads); labels stay on the host (they feed
the forest trainer, not the query step).
"""
from __future__ import annotations

import ctypes
import mmap
import os

import numpy as np

from . import _lib

LABEL_MAPS = {"reference": 0, "as_is": 1}
CHUNK_BYTES = 64 << 20


def _threads() -> int:
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:  # pragma: no cover
        return max(1, min(16, os.cpu_count() or 1))


def _chunks(buf, n_bytes: int, chunk_bytes: int):
    """Byte ranges [a, b) of ~chunk_bytes that start at line starts."""
    a = 0
    while a < n_bytes:
        b = min(n_bytes, a + chunk_bytes)
        if b < n_bytes:
            nl = buf.find(b"\n", b)
            b = n_bytes if nl < 0 else nl + 1
        yield a, b
        a = b


def _shape(addr: int, n: int, max_rows: int):
    rows, cols = ctypes.c_int64(), ctypes.c_int64()
    _lib.call("dal_text_shape", addr, n, int(max_rows), ctypes.addressof(rows), ctypes.addressof(cols))
    return rows.value, cols.value


def parse_labeled_text(path: str, n_samples=None, label_map: str = "reference"):
    """Host parse (no GPU): (X fp32 [N, D] numpy, y int64 [N]).  Bit-identical
    to ``np.array(fields, dtype=np.float64).astype(np.float32)`` per row."""
    X, y, _ = _load(path, n_samples, label_map, device=None)
    return X, y


def load_pool(path: str, n_samples=None, label_map: str = "reference", device=None,
              chunk_bytes: int = CHUNK_BYTES):
    """Parse the text file into pinned host chunks and upload them to HBM
    asynchronously.  Returns (x device fp32 [N, D], y int64 numpy [N]).
    The copies are ordered before any later work on the current stream."""
    from .engine import _require_cuda

    dev = _require_cuda(device)
    x, y, _ = _load(path, n_samples, label_map, device=dev, chunk_bytes=chunk_bytes)
    return x, y


def _load(path, n_samples, label_map, device, chunk_bytes: int = CHUNK_BYTES):
    if label_map not in LABEL_MAPS:
        raise ValueError(f"label_map must be one of {tuple(LABEL_MAPS)}")
    lm = LABEL_MAPS[label_map]
    max_rows = -1 if n_samples is None else int(n_samples)
    size = os.path.getsize(path)
    if size == 0:
        raise ValueError(f"{path}: empty file")
    with open(path, "rb") as fh:
        # a private (copy-on-write) mapping exposes an address to ctypes; its
        # pages are the file's page-cache pages (nothing is copied)
        mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_COPY)
    cbuf = (ctypes.c_char * size).from_buffer(mm)
    try:
        base = ctypes.addressof(cbuf)
        plan, total, cols = [], 0, None
        for a, b in _chunks(mm, size, chunk_bytes):
            if max_rows >= 0 and total >= max_rows:
                break
            r, c = _shape(base + a, b - a, -1 if max_rows < 0 else max_rows - total)
            if r == 0:
                continue
            if cols is None:
                cols = c
            elif c != cols:
                raise ValueError(f"{path}: rows with {c} and {cols} fields")
            plan.append((a, b, total, r))
            total += r
        if not plan:
            raise ValueError(f"{path}: no rows")
        if cols < 2:
            raise ValueError(f"{path}: need at least one feature and a label per row")
        d = cols - 1
        y = np.empty(total, dtype=np.int64)
        if device is None:
            X = np.empty((total, d), dtype=np.float32)
            for a, b, r0, r in plan:
                _lib.call("dal_parse_labeled_text", base + a, b - a, r, cols, lm,
                          X.ctypes.data + r0 * d * 4, y.ctypes.data + r0 * 8, _threads())
            return X, y, None
        return _upload(base, plan, total, d, cols, lm, y, device)
    finally:
        del cbuf
        mm.close()


def _upload(base, plan, total, d, cols, lm, y, device):
    import torch

    x = torch.empty((total, d), dtype=torch.float32, device=device)
    main = torch.cuda.current_stream(device)
    side = torch.cuda.Stream(device=device)
    side.wait_stream(main)  # x's allocation is ordered on main
    max_rows = max(r for _, _, _, r in plan)
    pinned = [torch.empty((max_rows, d), dtype=torch.float32, pin_memory=True) for _ in range(2)]
    done = [None, None]
    for i, (a, b, r0, r) in enumerate(plan):
        slot = i & 1
        if done[slot] is not None:
            done[slot].synchronize()  # the copy that last read this pinned buffer has finished
        buf = pinned[slot]
        _lib.call("dal_parse_labeled_text", base + a, b - a, r, cols, lm, buf.data_ptr(),
                  y.ctypes.data + r0 * 8, _threads())
        with torch.cuda.stream(side):
            x[r0:r0 + r].copy_(buf[:r], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        done[slot] = ev
    main.wait_stream(side)
    x.record_stream(side)
    for ev in done:
        if ev is not None:
            ev.synchronize()  # the pinned buffers are released after their copies
    return x, y, None


__all__ = ["parse_labeled_text", "load_pool"]
