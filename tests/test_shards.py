"""Preprocessed-shard writer / reader (preproc_dataset.py:59-84,
dataset.py:27-33): tar layout, round trip, shard rollover, brace lists, and
the reader's refusal to run code from a shard.  CPU only; the GPU writer
(write_preprocessed) is covered in test_gpu_shards.py."""
import io
import os
import pickle
import tarfile

import pytest
import torch


def _items(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(n):
        k = int(torch.randint(1, 300, (1,), generator=g))
        h, w = int(torch.randint(14, 900, (1,), generator=g)), int(torch.randint(14, 900, (1,), generator=g))
        out.append(dict(patches=torch.randn(k, 196, generator=g),
                        positions=torch.randint(0, 32, (k, 2), generator=g),
                        channels=torch.randint(0, 3, (k,), generator=g),
                        original_sizes=(h, w), patch_sizes=(h // 14, w // 14)))
    return out


def _write(shards, items, out, **kw):
    with shards.ShardWriter(os.path.join(out, "%06d.tar"), **kw) as w:
        for i, it in enumerate(items):
            w.write(shards.sample_of(i, it))
    return w.fnames


def _same(a, b):
    assert torch.equal(a["patches"], b["patches"])
    assert a["patches"].dtype == b["patches"].dtype
    assert torch.equal(a["positions"], b["positions"]) and b["positions"].dtype == torch.long
    assert torch.equal(a["channels"], b["channels"])
    assert tuple(a["original_sizes"]) == b["original_sizes"] and tuple(a["patch_sizes"]) == b["patch_sizes"]


@pytest.mark.parametrize("compress", [True, False])
def test_roundtrip_and_layout(pkg, tmp_path, compress):
    items = _items(7)
    names = _write(pkg.shards, items, str(tmp_path), compress=compress)
    assert [os.path.basename(n) for n in names] == ["000000.tar"]
    # member names / order of preproc_dataset.py:72-84 (webdataset: "<key>.<ext>")
    with tarfile.open(names[0], "r:gz" if compress else "r:") as tf:
        members = tf.getnames()
    exts = ["patches.pth", "positions.pth", "channels.pth", "original_size.pyd", "patch_size.pyd"]
    assert members == [f"{i:08}.{e}" for i in range(7) for e in exts]
    back = list(pkg.shards.load_preprocessed_dataset(str(tmp_path / "000000.tar")))
    assert len(back) == 7
    for a, b in zip(items, back):
        _same(a, b)


def test_rollover_and_brace_list(pkg, tmp_path):
    items = _items(20, seed=1)
    names = _write(pkg.shards, items, str(tmp_path), maxcount=6)
    assert len(names) == 4
    url = str(tmp_path / "0000{00..03}.tar")
    assert pkg.shards.braceexpand(url) == names
    back = list(pkg.shards.load_preprocessed_dataset(url))
    assert len(back) == 20
    for a, b in zip(items, back):
        _same(a, b)
    # a directory lists its shards in order
    assert len(list(pkg.shards.load_preprocessed_dataset(str(tmp_path)))) == 20
    # maxsize rollover (uncompressed payload bytes)
    d2 = tmp_path / "s"
    d2.mkdir()
    assert len(_write(pkg.shards, items, str(d2), maxsize=100_000)) > 1


def test_batched_dict_collate(pkg, tmp_path):
    items = _items(5, seed=2)
    _write(pkg.shards, items, str(tmp_path))
    bs = list(pkg.shards.batched(pkg.shards.load_preprocessed_dataset(str(tmp_path)), 2))
    assert [len(b["patches"]) for b in bs] == [2, 2, 1]
    assert set(bs[0]) == {"patches", "positions", "channels", "original_sizes", "patch_sizes"}


class _Evil:
    def __reduce__(self):
        return (os.getcwd, ())


def test_reader_refuses_code_in_shards(pkg, tmp_path):
    """.pyd members with globals (and non-weights .pth pickles) are skipped with a
    warning, never executed (warn_and_continue like dataset.py:30-32)."""
    items = _items(2, seed=3)
    s0 = pkg.shards.sample_of(0, items[0])
    s1 = pkg.shards.sample_of(1, items[1])
    s1["original_size.pyd"] = pickle.dumps(_Evil())
    with pkg.shards.ShardWriter(str(tmp_path / "%06d.tar")) as w:
        w.write(s0)
        w.write(s1)
    with pytest.warns(UserWarning, match="refused"):
        back = list(pkg.shards.load_preprocessed_dataset(str(tmp_path)))
    assert len(back) == 1
    _same(items[0], back[0])
    b = io.BytesIO()
    torch.save({"x": _Evil()}, b)
    with pytest.raises(Exception):
        pkg.shards.decode_sample({**s0, "patches.pth": b.getvalue()})
