"""Data layer: calendar rules, synthetic generator, featurizers, split, CSV, HTML (CPU)."""
import datetime as dt
import os

import numpy as np
import pytest

from euromillioner_amd.data import synthetic as syn
from euromillioner_amd.data.draws import (DrawSet, featurize_raw, lag_features, mask_bits, multi_hot,
                                          positional_split)

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def test_calendar_matches_reference_range():
    d = syn.draw_dates()
    assert str(d[0]) == "2004-02-13" and str(d[-1]) == "2020-06-12"
    assert len(d) == 1328  # ~1,328 draws up to 2020-06-14
    wd = (d.astype("int64") + 3) % 7  # Mon=0
    before = d < np.datetime64("2011-05-10")
    assert set(wd[before]) == {4}  # Fridays only
    assert set(wd[~before]) == {1, 4}  # Tuesdays and Fridays


def test_fast_calendar_equals_slow():
    assert np.array_equal(syn.draw_dates(n=3000), syn.draw_dates_fast(3000))


def test_star_ranges_by_era():
    d = np.array(["2011-05-06", "2011-05-10", "2016-09-23", "2016-09-27"], dtype="datetime64[D]")
    assert list(syn.star_max_for(d)) == [9, 11, 11, 12]


def test_synthetic_rules_and_determinism():
    ds = DrawSet.synthetic(seed=3, planted=0.5)
    ds.validate()
    sm = syn.star_max_for(ds.dates)
    assert (ds.numbers[:, 5:7].max(1) <= sm).all()
    assert (np.diff(ds.numbers[:, :5].astype(int), axis=1) > 0).all()  # sorted, distinct
    ds2 = DrawSet.synthetic(seed=3, planted=0.5)
    assert np.array_equal(ds.numbers, ds2.numbers)


@pytest.mark.parametrize("planted", [0.0, 0.3, 1.0])
def test_native_generator_bit_identical_to_python(planted):
    sm = syn.star_max_for(syn.draw_dates(n=700))
    a, pa = syn.generate_draws_py(700, seed=11, planted=planted, star_max=sm)
    b, pb = syn.generate_draws(700, seed=11, planted=planted, star_max=sm, native=True)
    assert np.array_equal(a, b) and np.array_equal(pa, pb)


def test_planted_structure_is_present():
    nums, perm = syn.generate_draws(20000, seed=1, planted=0.9, native=True)
    pim = perm[:50]
    hits = 0
    for t in range(len(nums) - 1):
        nxt = set(nums[t + 1, :5])
        hits += sum(pim[n - 1] in nxt for n in nums[t, :5])
    assert hits / (5 * (len(nums) - 1)) > 0.85
    iid, _ = syn.generate_draws(20000, seed=1, planted=0.0, native=True)
    freq = np.bincount(iid[:, :5].reshape(-1), minlength=51)[1:] / (5 * len(iid))
    assert np.allclose(freq, 1 / 50, atol=0.004)


def test_featurize_raw_matches_reference_columns():
    ds = DrawSet.synthetic(seed=0).slice(0, 3)
    raw = featurize_raw(ds)
    # 2004-02-13 is a Friday: ISO dayOfWeek 5 (Main.java:94 getDayOfWeek().getValue())
    assert list(raw[0, :4]) == [5, 2, 13, 2004]
    assert raw.shape == (3, 11)
    assert np.array_equal(raw[:, 4:], ds.numbers[:, :7])


def test_multi_hot_and_masks_agree():
    ds = DrawSet.synthetic(seed=2).slice(0, 50)
    mh = multi_hot(ds.numbers)
    assert (mh.sum(1) == 7).all()
    m = mask_bits(ds.numbers)
    for i in range(50):
        bits = [b for b in range(64) if (int(m[i]) >> b) & 1]
        assert bits == list(np.nonzero(mh[i])[0])


def test_lag_features():
    ds = DrawSet.synthetic(seed=2).slice(0, 10)
    X, Y = lag_features(ds.numbers, lags=3)
    assert X.shape == (7, 186) and Y.shape == (7, 62)
    assert np.array_equal(X[0, 124:], multi_hot(ds.numbers[2:3])[0])
    assert np.array_equal(Y[0], multi_hot(ds.numbers[3:4])[0])


def test_positional_split_is_int_of_70_percent():
    for n in (0, 1, 10, 1328, 1329):
        assert positional_split(n) == int(0.7 * n)


def test_csv_roundtrip(tmp_path):
    from euromillioner_amd.data.csv_io import read_draws_csv, write_draws_csv

    ds = DrawSet.synthetic(seed=5).slice(0, 40)
    p = tmp_path / "d.csv"
    write_draws_csv(str(p), ds)
    text = p.read_text()
    assert text.count("\n") == 41 and text.startswith("date,day_of_week")
    back = read_draws_csv(str(p))
    assert np.array_equal(back.numbers, ds.numbers) and np.array_equal(back.dates, ds.dates)


def test_reference_csv_byte_format(tmp_path):
    from euromillioner_amd.data.csv_io import (REFERENCE_HEADER, read_reference_csv,
                                               reference_records_to_drawset, write_reference_csv)

    ds = DrawSet.synthetic(seed=5).slice(0, 10)
    tr, va = tmp_path / "emn.csv", tmp_path / "emn_validation.csv"
    margin = write_reference_csv(str(tr), str(va), ds)
    assert margin == 7
    t = tr.read_text()
    assert "\n" not in t and t.startswith(REFERENCE_HEADER) and t.endswith(", ")  # defect D-b reproduced
    rec = read_reference_csv(str(tr))
    assert rec.shape == (7, 11)
    back = reference_records_to_drawset(np.concatenate([rec, read_reference_csv(str(va))]))
    assert np.array_equal(back.numbers, ds.numbers)


def test_native_numeric_csv_loader(tmp_path):
    from euromillioner_amd.data.csv_io import load_numeric_csv

    p = tmp_path / "m.csv"
    p.write_text("a,b,c\n1, 2.5, 3,\n4,x,6\n\n7,8\n")
    X, y = load_numeric_csv(str(p), skip_header=True, label_column=0)
    assert list(y) == [1, 4, 7]
    assert X.shape == (3, 2)
    assert X[0, 0] == 2.5 and np.isnan(X[1, 0]) and np.isnan(X[2, 1])


def test_html_fixture_parses():
    from euromillioner_amd.data.html_table import parse_results_table

    html = open(os.path.join(FIX, "results_table.html")).read()
    ds = parse_results_table(html)
    ref = DrawSet.synthetic(seed=7).slice(0, 12)
    assert len(ds) == 12  # info row dropped (Main.java:66-67)
    assert np.array_equal(ds.numbers, ref.numbers) and np.array_equal(ds.dates, ref.dates)


def test_html_missing_table_raises():
    from euromillioner_amd.data.html_table import parse_results_table

    with pytest.raises(ValueError):
        parse_results_table("<html><table class='other'><tr><td>x</td></tr></table></html>")


def test_html_date_format_english():
    from euromillioner_amd.data.html_table import parse_date

    assert parse_date("Fri, Jun 12, 2020") == dt.date(2020, 6, 12)
    assert parse_date("Tue,  May 10, 2011") == dt.date(2011, 5, 10)


def test_csv_header_flag(tmp_path):
    from euromillioner_amd.data.csv_io import read_draws_csv

    p = tmp_path / "h.csv"
    p.write_text("5,1,3,2020,1,2,3,4,5,6,7\n4,2,4,2020,8,9,10,11,12,1,2\n")
    assert len(read_draws_csv(str(p))) == 2  # detected: no header
    assert len(read_draws_csv(str(p), header=True)) == 1  # forced: first row is a header
    assert len(read_draws_csv(str(p), header=False)) == 2
