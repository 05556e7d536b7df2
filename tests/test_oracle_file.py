"""CPU: the file-backed restatement of config 1 (ora_sst_decode_file: the
reference's unbuffered *os.File decode, one read(2) per field,
sstable.go:87-127,214-268) agrees with the in-memory oracle (ora_sst_decode)
on the pair count of intact images and on which damaged images fail."""
import numpy as np

import pyoracle as ora
from lsmgpu import synth


def _image(n):
    keys, koff, vals, voff = synth.kv_stream(n)
    img, _ = ora.build_sst(keys, koff, vals, voff, 0, n)
    return img


def test_file_decode_matches_memory_decode(tmp_path):
    for n in (1, 7, 15_888):                       # 15,888: config 1's 2,297,320-byte file
        img = _image(n)
        p = tmp_path / f"f{n}.sst"
        p.write_bytes(img.tobytes())
        rc, meta, *_ = ora.sst_decode(img)
        assert meta.stage == 0 and meta.nidx == n
        assert ora.sst_decode_file(str(p)) == n
    assert _image(15_888).size == 2_297_320


def test_file_decode_failures_agree(tmp_path):
    img = _image(300)
    rng = np.random.default_rng(3)
    cases = [img[:-1], img[:-40], img[:10], img[:0]]
    for _ in range(20):                            # bytes flipped in the framing / regions
        b = img.copy()
        at = int(rng.integers(0, b.size))
        b[at] ^= 0xFF
        cases.append(b)
    for i, b in enumerate(cases):
        p = tmp_path / f"c{i}.sst"
        p.write_bytes(b.tobytes())
        rc, meta, *_ = ora.sst_decode(b)
        got = ora.sst_decode_file(str(p))
        if meta.stage == 0:   # GetKeyValuePairs: (nil, nil) when either side is empty
            assert got == (meta.nidx if meta.nidx and meta.ndata else 0), i
        else:
            assert got < 0, (i, meta.stage, got)
