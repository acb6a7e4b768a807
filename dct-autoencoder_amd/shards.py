"""Preprocessed-shard writer / reader.

Reference: preproc_dataset.py:59-84 writes, through webdataset's
ShardWriter(output_dir + "/%06d.tar", maxsize=1e9, compress=True), one sample
per image with the members

    {key}.patches.pth      torch.save of the (k, P*P) spectral tokens
    {key}.positions.pth    torch.save of the (k, 2) int64 [h, w] positions
    {key}.channels.pth     torch.save of the (k,) int64 channels
    {key}.original_size.pyd  pickle of the (h, w) tuple
    {key}.patch_size.pyd     pickle of the (ph, pw) tuple

(key = f"{i:08}"), and dataset.py:27-33 reads them back as dicts with the
keys of FE.preprocess (patches, positions, channels, original_sizes,
patch_sizes).  webdataset is not a dependency here: the tar layout above is
written and read with the standard library, byte-compatible in the members
that matter (gzip-compressed tar stream, member order per sample as the
reference's dict order).

The writer takes its tokens from the GPU feature path
(DCTAutoencoderFeatureExtractor.preprocess_many: one launch sequence per
batch of images) and overlaps the device->host copy + serialisation of batch
i with the GPU work of batch i+1 (a writer thread).

The reader never executes code from a shard: ``.pth`` members go through
``torch.load(weights_only=True)`` and ``.pyd`` members through an unpickler
that refuses every global (a tuple of ints needs none).
"""
from __future__ import annotations

import glob
import io
import os
import pickle
import queue
import re
import tarfile
import threading
import time
from typing import Dict, Iterable, Iterator, List, Optional, Sequence

import torch

FIELDS = (("patches", "patches.pth"), ("positions", "positions.pth"), ("channels", "channels.pth"),
          ("original_sizes", "original_size.pyd"), ("patch_sizes", "patch_size.pyd"))


# ---- serialisation (webdataset's default encoders for .pth / .pyd) ----------


def _pth_bytes(t: torch.Tensor) -> bytes:
    b = io.BytesIO()
    torch.save(t, b)
    return b.getvalue()


def _pyd_bytes(v) -> bytes:
    return pickle.dumps(v)


class _NoGlobalsUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        raise pickle.UnpicklingError(f".pyd member references {module}.{name}: refused (plain data only)")


def _pyd_load(b: bytes):
    v = _NoGlobalsUnpickler(io.BytesIO(b)).load()
    return tuple(v) if isinstance(v, list) else v


def _pth_load(b: bytes) -> torch.Tensor:
    return torch.load(io.BytesIO(b), map_location="cpu", weights_only=True)


# ---- writer ------------------------------------------------------------------


class ShardWriter:
    """webdataset.ShardWriter subset: ``pattern % shard`` files, a new shard
    once ``maxsize`` bytes (uncompressed payload) or ``maxcount`` samples are
    reached, gzip-compressed tar streams when ``compress``."""

    def __init__(self, pattern: str, maxsize: float = 1e9, maxcount: int = 100000, compress: bool = True,
                 start_shard: int = 0):
        self.pattern = pattern
        self.maxsize = maxsize
        self.maxcount = maxcount
        self.compress = compress
        self.shard = start_shard
        self.tar: Optional[tarfile.TarFile] = None
        self.fileobj = None
        self.size = 0
        self.count = 0
        self.total = 0
        self.fnames: List[str] = []

    def _next(self):
        self.close()
        fname = self.pattern % self.shard
        self.shard += 1
        self.fileobj = open(fname, "wb")
        self.tar = tarfile.open(fileobj=self.fileobj, mode="w|gz" if self.compress else "w|")
        self.fnames.append(fname)
        self.size = 0
        self.count = 0

    def write(self, sample: Dict):
        """sample: {"__key__": str, "<ext>": bytes | tensor | tuple ...}"""
        if self.tar is None or self.size >= self.maxsize or self.count >= self.maxcount:
            self._next()
        key = sample["__key__"]
        now = time.time()
        for ext, v in sample.items():
            if ext == "__key__":
                continue
            if isinstance(v, (bytes, bytearray)):
                data = bytes(v)
            elif ext.endswith(".pth"):
                data = _pth_bytes(v)
            elif ext.endswith(".pyd"):
                data = _pyd_bytes(v)
            else:
                raise ValueError(f"no encoder for {ext}")
            ti = tarfile.TarInfo(f"{key}.{ext}")
            ti.size = len(data)
            ti.mtime = now
            ti.mode = 0o444
            ti.uname = ti.gname = "bigdata"
            self.tar.addfile(ti, io.BytesIO(data))
            self.size += len(data)
        self.count += 1
        self.total += 1

    def close(self):
        if self.tar is not None:
            self.tar.close()
            self.fileobj.close()
        self.tar = None
        self.fileobj = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def sample_of(i: int, item: Dict) -> Dict:
    """One preprocess() dict -> the reference's shard sample (preproc_dataset.py:66-84)."""
    s = {"__key__": f"{i:08}"}
    for field, ext in FIELDS:
        v = item[field]
        s[ext] = v.cpu() if torch.is_tensor(v) else tuple(int(t) for t in v)
    return s


def write_preprocessed(fe, images: Iterable[torch.Tensor], output_dir: str, batch: int = 64,
                       maxsize: float = 1e9, compress: bool = True, dtype: Optional[torch.dtype] = None,
                       start_index: int = 0) -> List[str]:
    """preproc_dataset.main without the dataset plumbing: ``images`` yields
    (3, h, w) RGB tensors in [0, 1]; each chunk of ``batch`` images runs
    through ``fe.preprocess_many`` on the GPU, its tokens come back to the
    host in one copy per field and a writer thread serialises them while the
    GPU works on the next chunk.  Returns the shard file names."""
    os.makedirs(output_dir, exist_ok=True)
    q: "queue.Queue" = queue.Queue(maxsize=2)
    err: List[BaseException] = []
    writer = ShardWriter(os.path.join(output_dir, "%06d.tar"), maxsize=maxsize, compress=compress)

    def drain():
        try:
            while True:
                job = q.get()
                if job is None:
                    return
                first, items, ev = job
                ev.synchronize()
                for j, it in enumerate(items):
                    writer.write(sample_of(first + j, it))
        except BaseException as e:  # surfaced in the producer
            err.append(e)
            while q.get() is not None:
                pass

    th = threading.Thread(target=drain, daemon=True)
    th.start()

    def flush(chunk, first):
        outs = fe.preprocess_many(chunk)
        host = []
        for it in outs:
            h = dict(it)
            pt = it["patches"] if dtype is None else it["patches"].to(dtype)
            h["patches"] = pt.to("cpu", non_blocking=True)
            h["positions"] = it["positions"].to("cpu", non_blocking=True)
            h["channels"] = it["channels"].to("cpu", non_blocking=True)
            host.append(h)
        ev = torch.cuda.Event()
        ev.record()
        q.put((first, host, ev))

    i = start_index
    chunk: List[torch.Tensor] = []
    try:
        for im in images:
            if err:
                break
            chunk.append(im)
            if len(chunk) == batch:
                flush(chunk, i)
                i += len(chunk)
                chunk = []
        if chunk and not err:
            flush(chunk, i)
    finally:
        q.put(None)
        th.join()
        writer.close()
    if err:
        raise err[0]
    return writer.fnames


# ---- reader ------------------------------------------------------------------


def braceexpand(url: str) -> List[str]:
    """'000{000..430}.tar' -> the 431 names (webdataset's shard-list syntax)."""
    m = re.search(r"\{(\d+)\.\.(\d+)\}", url)
    if not m:
        return [url]
    a, b = m.group(1), m.group(2)
    width = len(a)
    return [n for v in range(int(a), int(b) + 1)
            for n in braceexpand(url[:m.start()] + str(v).zfill(width) + url[m.end():])]


def _urls(spec) -> List[str]:
    if isinstance(spec, (list, tuple)):
        return [u for s in spec for u in _urls(s)]
    if os.path.isdir(spec):
        return sorted(glob.glob(os.path.join(spec, "*.tar")))
    return braceexpand(spec)


def _open_tar(path: str) -> tarfile.TarFile:
    with open(path, "rb") as f:
        gz = f.read(2) == b"\x1f\x8b"
    return tarfile.open(path, mode="r|gz" if gz else "r|")


def iter_samples(spec) -> Iterator[Dict]:
    """Raw samples {"__key__", "<ext>": bytes} grouped by key, in tar order."""
    for path in _urls(spec):
        tf = _open_tar(path)
        cur: Optional[Dict] = None
        for ti in tf:
            if not ti.isfile():
                continue
            base = os.path.basename(ti.name)
            key, _, ext = base.partition(".")
            data = tf.extractfile(ti).read()
            if cur is None or cur["__key__"] != key:
                if cur is not None:
                    yield cur
                cur = {"__key__": key, "__url__": path}
            cur[ext] = data
        if cur is not None:
            yield cur
        tf.close()


def decode_sample(s: Dict) -> Dict:
    """dataset.py:31-32: the FE.preprocess dict of one shard sample."""
    out = {}
    for field, ext in FIELDS:
        if ext not in s:
            raise KeyError(f"sample {s.get('__key__')} has no {ext}")
        out[field] = _pth_load(s[ext]) if ext.endswith(".pth") else _pyd_load(s[ext])
    return out


def load_preprocessed_dataset(dataset_url) -> Iterator[Dict]:
    """dataset.py:27-33: iterate the decoded samples of a shard list (brace
    syntax, a directory, or a list of paths).  Samples that fail to decode
    are skipped with a warning, like webdataset's warn_and_continue."""
    import warnings
    for s in iter_samples(dataset_url):
        try:
            yield decode_sample(s)
        except Exception as e:  # noqa: BLE001  (warn_and_continue)
            warnings.warn(f"skipping sample {s.get('__key__')} of {s.get('__url__')}: {e}")


def dict_collate(x: Sequence[Dict]) -> Dict[str, list]:
    """dataset.py:8-15."""
    assert len(x) > 0
    cols = x[0].keys()
    return {k: [row[k] for row in x] for k in cols}


def batched(samples: Iterable[Dict], batch_size: int) -> Iterator[Dict[str, list]]:
    """DataLoader(batch_size, collate_fn=dict_collate) over an iterable dataset."""
    buf: List[Dict] = []
    for s in samples:
        buf.append(s)
        if len(buf) == batch_size:
            yield dict_collate(buf)
            buf = []
    if buf:
        yield dict_collate(buf)
