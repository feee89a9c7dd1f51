"""Pool ingest: the native text parser against the
reference's own parsing semantics -- uncertainty_sampling.py:37-42
``LabeledPoint(0 if int(_[-1]) == -1 else 1, np.array(_[:-1]).astype(float))``
and density_weighting.py:59-65 ``take(n_samples)`` -- restated in Python
below (fp64 parse, narrowed to the fp32 pool), on the reference's bundled data
(the checkerboard fixtures and unlabeled_init) and on ragged / signed /
scientific-notation inputs."""
import os

import numpy as np
import pytest

from conftest import load_golden


def _ref_parse(path, n_samples=None, label_map="reference"):
    rows = []
    for line in open(path):
        parts = line.strip().split()
        if not parts:
            continue
        rows.append(parts)
        if n_samples is not None and len(rows) >= n_samples:
            break
    X = np.array([r[:-1] for r in rows]).astype(float).astype(np.float32)
    lab = [int(r[-1]) for r in rows]
    y = np.array([0 if v == -1 else 1 for v in lab] if label_map == "reference" else lab, dtype=np.int64)
    return X, y


def _write(tmp_path, name, X, y, fmt="%r", sep=" "):
    p = tmp_path / name
    with open(p, "w") as fh:
        for i in range(X.shape[0]):
            fh.write(sep.join(fmt % float(v) for v in X[i]) + sep + str(int(y[i])) + "\n")
    return str(p)


def test_parse_checkerboard_fixture(tmp_path):
    from dal.ingest import parse_labeled_text

    g = load_golden("checkerboard2x2.npz")
    X, y = g["X"].astype(np.float64), g["y"]
    p = _write(tmp_path, "cb.txt", X, y)
    got_x, got_y = parse_labeled_text(p, label_map="as_is")
    ref_x, ref_y = _ref_parse(p, label_map="as_is")
    assert np.array_equal(got_x.view(np.int32), ref_x.view(np.int32))
    assert np.array_equal(got_y, ref_y)


def test_parse_striatum_style_labels_and_take(tmp_path):
    from dal.ingest import parse_labeled_text

    rng = np.random.default_rng(4)
    X = rng.standard_normal((5000, 17)) * 10.0 ** rng.integers(-8, 8, size=(5000, 17))
    y = rng.choice([-1, 1], size=5000)
    p = _write(tmp_path, "s.txt", X, y, fmt="%.17g", sep="\t")
    for n in (None, 1, 4321):
        got_x, got_y = parse_labeled_text(p, n_samples=n)
        ref_x, ref_y = _ref_parse(p, n_samples=n)
        assert np.array_equal(got_x.view(np.int32), ref_x.view(np.int32))
        assert np.array_equal(got_y, ref_y)
        assert set(np.unique(got_y)) <= {0, 1}


def test_parse_double_rounding_matches_fp64_then_fp32(tmp_path):
    """Decimal strings halfway between fp32 neighbours after fp64 rounding:
    strtod + narrow gives the fp64-first bits the reference's astype(float)
    then the fp32 pool would hold."""
    from dal.ingest import parse_labeled_text

    vals = ["1.00000005960464477539", "1.0000000596046448", "0.1", "-3.4028235677973366e+38",
            "1e-45", "7.006492321624086e-46", "16777217", "0", "-0", "2.5e-08"]
    p = tmp_path / "r.txt"
    p.write_text("\n".join(f"{v} {v} 1" for v in vals) + "\n\n   \n")
    got_x, got_y = parse_labeled_text(str(p))
    ref_x, _ = _ref_parse(str(p))
    assert np.array_equal(got_x.view(np.int32), ref_x.view(np.int32))
    assert got_y.tolist() == [1] * len(vals)


def test_parse_rejects_tokens_python_float_rejects(tmp_path):
    """Hex floats and nan(chars) parse with strtod but raise in the
    reference's float(); inf/nan spellings float() takes are accepted."""
    from dal import _lib
    from dal.ingest import parse_labeled_text

    p = tmp_path / "hex.txt"
    for tok in ("0x1p3", "-0X10", "nan(123)"):
        with pytest.raises(ValueError):
            float(tok)
        p.write_text(f"1 {tok} 1\n")
        with pytest.raises(_lib.DalError):
            parse_labeled_text(str(p))
    p.write_text("inf -Infinity 1\nNaN +1.5 -1\n")
    got_x, got_y = parse_labeled_text(str(p))
    ref_x, ref_y = _ref_parse(str(p))
    assert np.array_equal(got_x.view(np.int32), ref_x.view(np.int32))
    assert np.array_equal(got_y, ref_y)


def test_parse_digit_group_underscores_like_python(tmp_path):
    """PEP 515 underscores between digits parse as the reference's
    astype(float) / int() read them; any other underscore rejects the token."""
    from dal import _lib
    from dal.ingest import parse_labeled_text

    p = tmp_path / "us.txt"
    p.write_text("1_000.5 2_5e1_0 1\n1e1_0 -0_5 1_0\n")
    got_x, got_y = parse_labeled_text(str(p))
    ref_x, ref_y = _ref_parse(str(p))
    assert np.array_equal(got_x.view(np.int32), ref_x.view(np.int32))
    assert np.array_equal(got_y, ref_y)
    for tok in ("1__0", "_1", "1_", "1_.5", "1._5", "1_e5"):
        with pytest.raises(ValueError):
            float(tok)
        p.write_text(f"1 {tok} 1\n")
        with pytest.raises(_lib.DalError):
            parse_labeled_text(str(p))


def test_parse_ignores_process_numeric_locale(tmp_path):
    """Python float() ignores LC_NUMERIC; so does the native parser (a
    comma-decimal locale must not break '0.5')."""
    import locale

    from dal.ingest import parse_labeled_text

    p = tmp_path / "loc.txt"
    p.write_text("0.5 1.25 1\n")
    old = locale.setlocale(locale.LC_NUMERIC)
    switched = False
    for name in ("de_DE.UTF-8", "de_DE.utf8", "fr_FR.UTF-8", "fr_FR.utf8"):
        try:
            locale.setlocale(locale.LC_NUMERIC, name)
            switched = True
            break
        except locale.Error:
            continue
    if not switched:
        pytest.skip("no comma-decimal locale installed in this image (locale -a: C, C.utf8, POSIX)")
    try:
        assert locale.localeconv()["decimal_point"] == ","
        got_x, _ = parse_labeled_text(str(p))
    finally:
        locale.setlocale(locale.LC_NUMERIC, old)
    assert got_x.tolist() == [[0.5, 1.25]]


def test_parse_rejects_ragged_and_bad_fields(tmp_path):
    from dal import _lib
    from dal.ingest import parse_labeled_text

    p = tmp_path / "bad.txt"
    p.write_text("1 2 3 1\n4 5 1\n")
    with pytest.raises((ValueError, _lib.DalError)):
        parse_labeled_text(str(p))
    p.write_text("1 2 x 1\n")
    with pytest.raises(_lib.DalError):
        parse_labeled_text(str(p))
    p.write_text("1 2 3 1.5\n")  # int('1.5') raises in the reference
    with pytest.raises(_lib.DalError):
        parse_labeled_text(str(p))


def test_parse_large_multithreaded_chunks(tmp_path):
    from dal import ingest

    rng = np.random.default_rng(9)
    X = rng.random((60000, 12)).astype(np.float32).astype(np.float64)
    y = rng.choice([-1, 1], size=60000)
    p = _write(tmp_path, "big.txt", X, y)
    ref_x, ref_y = _ref_parse(p)
    got_x, got_y, _ = ingest._load(p, None, "reference", None, chunk_bytes=1 << 18)
    assert np.array_equal(got_x, ref_x) and np.array_equal(got_y, ref_y)
    got_x, got_y, _ = ingest._load(p, 33333, "reference", None, chunk_bytes=1 << 18)
    assert np.array_equal(got_x, ref_x[:33333]) and np.array_equal(got_y, ref_y[:33333])


@pytest.mark.gpu
def test_load_pool_pinned_upload_and_select(cuda, tmp_path):
    """Parse into pinned chunks + async H2D upload, then the GPU query step on
    the uploaded pool equals the oracle on the reference-parsed pool."""
    from dal import ingest
    from dal import uncertainty_sampling as us
    from dal.forest import Forest
    from oracle import dal_oracle as O

    rng = np.random.default_rng(5)
    X = rng.random((70000, 16))
    y = rng.choice([-1, 1], size=70000)
    p = _write(tmp_path, "pool.txt", X, y, fmt="%.9g")
    x_dev, got_y = ingest._load(p, None, "reference", cuda, chunk_bytes=1 << 20)[:2]
    ref_x, ref_y = _ref_parse(p)
    assert np.array_equal(x_dev.cpu().numpy().view(np.int32), ref_x.view(np.int32))
    assert np.array_equal(got_y, ref_y)
    F = Forest.synthetic(10, 4, 16, seed=1)
    of = O.synthetic_forest(10, 4, 16, seed=1)
    unl = np.arange(10, 70000)
    sel = us.select(x_dev, unl, F, 50, device=cuda)
    _, ref_idx, _ = O.uncertainty_select(ref_x, unl, of, 50)
    assert np.array_equal(sel.indices.cpu().numpy(), ref_idx)


def test_parse_long_tokens_huge_labels_and_nul(tmp_path):
    """Tokens longer than the parser's stack buffer, labels beyond int64 and
    embedded NUL bytes read as the reference's float() / int() read them
    (NUL: rejected; a huge label is not -1 -> 1)."""
    from dal import _lib
    from dal.ingest import parse_labeled_text

    p = tmp_path / "long.txt"
    p.write_text("1 " + "9" * 200 + " 1\n" + "1_" * 150 + "1 2 " + "9" * 80 + "\n3 4 -" + "0" * 70 + "1\n")
    got_x, got_y = parse_labeled_text(str(p))
    ref_x, ref_y = _ref_parse(str(p))
    assert np.array_equal(got_x.view(np.int32), ref_x.view(np.int32))
    assert np.array_equal(got_y, ref_y)
    for text in ("1 2\x00abc 1\n", "1 2 1\x00\n"):
        p.write_bytes(text.encode())
        with pytest.raises(_lib.DalError):
            parse_labeled_text(str(p))
