"""CPU: speq::file_to_map grammar (/root/reference/src/file_to_map.cpp:20-119) through the C ABI."""
import os

import pytest

from speq_amd import SpeqError, file_to_map
from speq_amd._lib import SPEQ_E_ARG, SPEQ_E_IO

HERE = os.path.dirname(os.path.abspath(__file__))


def _write(tmp_path, text, name="g.txt"):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_reference_fixture_without_counts_is_rejected():
    """The reference's only fixture (test/genome_groupings.txt, copied as data) has no "(count)": the reference's
    std::stoi throws std::invalid_argument (file_to_map.cpp:43). We fail the same way, with a clear message."""
    with pytest.raises(SpeqError) as e:
        file_to_map(os.path.join(HERE, "golden", "genome_groupings.txt"))
    assert e.value.code == SPEQ_E_ARG
    assert "(count)" in str(e.value)


def test_reference_fixture_with_counts():
    g = file_to_map(os.path.join(HERE, "golden", "genome_groupings_counted.txt"))
    assert g.names == ["MCV-1p", "MCV-1va", "MCV-1vb1", "MCV-1vb2", "MCV-1vc", "MCV-1vd", "MCV-2", "MCV-2v",
                       "MCV-3", "MCV-4", "Homo sapiens", "Human herpesvirus 5", "Human papillomavirus 5/16"]
    assert g.counts == [8, 14, 2, 2, 1, 1, 8, 1, 1, 3, 639, 1, 2]
    s = g.scaffolds
    assert len(s) == 683
    assert s[0:6] == [0] * 6 and s[36] == 0 and s[37] == 0
    assert s[6:19] == [1] * 13 and s[38] == 1
    assert s[19] == 2 and s[20] == 2 and s[21:23] == [3, 3] and s[39] == 4 and s[23] == 5
    assert s[24:31] == [6] * 7 and s[40] == 6 and s[31] == 7 and s[32] == 8 and s[33:36] == [9] * 3
    assert s[41:680] == [10] * 639 and s[680] == 11 and s[681:683] == [12, 12]
    assert g.errors == ""


def test_comments_gaps_and_later_lines_win(tmp_path):
    p = _write(tmp_path, "# full comment\nA(2): 0, 3  # inline: 9\nno colon here\nB(1): 3-4\n")
    g = file_to_map(p)
    assert g.names == ["A", "B"] and g.counts == [2, 1]
    assert g.scaffolds == [0, -1, -1, 1, 1]  # gaps are -1; index 3 reassigned by the later line


def test_bad_tokens_are_reported_and_skipped(tmp_path):
    p = _write(tmp_path, "A(1): 0, x, 2-y, ,1\n")
    g = file_to_map(p)
    assert g.scaffolds == [0, 0]
    assert "A non-integer index was detected and ignored at: x" in g.errors
    assert "A non-integer range was detected and ignored at: 2-y" in g.errors
    assert g.errors.count("Error in parsing groupings line: A(1): 0, x, 2-y, ,1") == 3


def test_name_is_untrimmed_and_whitespace_inside_tokens(tmp_path):
    p = _write(tmp_path, "Homo sapiens (3):\t0 - 2 ,\t 5\n")
    g = file_to_map(p)
    assert g.names == ["Homo sapiens "] and g.counts == [3]
    assert g.scaffolds == [0, 0, 0, -1, -1, 0]


def test_missing_file(tmp_path):
    with pytest.raises(SpeqError) as e:
        file_to_map(str(tmp_path / "nope.txt"))
    assert e.value.code == SPEQ_E_IO
