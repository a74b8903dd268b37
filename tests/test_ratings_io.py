"""mf_read_ratings: CSV (Flink readCsvFile default), MovieLens u.data (tabs + timestamp), auto
delimiter, header skip, blank lines, errors, and a multi-chunk file against numpy."""
import numpy as np
import pytest

import mfhip


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_csv_default_delimiter(tmp_path):
    p = write(tmp_path, "r.csv", "1,2,3.5\n-4,5,1e-3\n\n7,8,2\n")
    u, i, r = mfhip.read_ratings(p)
    assert u.tolist() == [1, -4, 7] and i.tolist() == [2, 5, 8]
    assert r.tolist() == [3.5, 1e-3, 2.0]


def test_movielens_udata_tabs_and_timestamp(tmp_path):
    p = write(tmp_path, "u.data", "196\t242\t3\t881250949\n186\t302\t3\t891717742\r\n22\t377\t1\t878887116")
    u, i, r = mfhip.read_ratings(p, delimiter="\t")
    assert u.tolist() == [196, 186, 22] and i.tolist() == [242, 302, 377] and r.tolist() == [3.0, 3.0, 1.0]


def test_auto_delimiter_and_header(tmp_path):
    p = write(tmp_path, "r.txt", "user item rating\n1  2 3\n4,\t5, 6.25\n")
    u, i, r = mfhip.read_ratings(p, delimiter="", skip_lines=1)
    assert u.tolist() == [1, 4] and i.tolist() == [2, 5] and r.tolist() == [3.0, 6.25]


def test_bad_line_names_the_line(tmp_path):
    p = write(tmp_path, "bad.csv", "1,2,3\n4,x,5\n")
    with pytest.raises(mfhip.MFError, match="line 2"):
        mfhip.read_ratings(p)
    with pytest.raises(mfhip.MFError, match="cannot open"):
        mfhip.read_ratings(str(tmp_path / "missing.csv"))


def test_empty_file(tmp_path):
    u, i, r = mfhip.read_ratings(write(tmp_path, "e.csv", ""))
    assert len(u) == len(i) == len(r) == 0


def test_large_file_matches_numpy(tmp_path):
    rng = np.random.default_rng(0)
    n = 300_000
    u = rng.integers(-2**31, 2**31 - 1, n)
    i = rng.integers(0, 10**6, n)
    r = np.round(rng.uniform(0, 5, n), 3)
    p = tmp_path / "big.csv"
    with open(p, "w") as f:
        for a, b, c in zip(u, i, r):
            f.write(f"{a},{b},{c}\n")
    gu, gi, gr = mfhip.read_ratings(str(p))
    assert np.array_equal(gu, u.astype(np.int32)) and np.array_equal(gi, i) and np.array_equal(gr, r)
