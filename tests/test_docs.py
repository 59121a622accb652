"""The integration guide keeps the warnings a kuma maintainer needs (VERDICT
r05 #4): the synchronous member swap alone regresses kuma's client and is
supported only with TxLoop; KMWS_ERR_TIMEOUT retires the resident grid for the
whole process; loop threads map to GPUs by the device policy."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def section(text: str, title: str) -> str:
    i = text.index(title)
    j = text.find("\n### ", i + len(title))
    k = text.find("\n## ", i + len(title))
    ends = [x for x in (j, k) if x > 0]
    return text[i:min(ends) if ends else len(text)]


def norm(s: str) -> str:
    return re.sub(r"\s+", " ", re.sub(r"\n> ?", "\n", s))


def test_member_swap_is_not_a_standalone_step():
    s = norm(section(open(os.path.join(ROOT, "INTEGRATION.md")).read(), "### 3.1 The member swap"))
    assert "Not a standalone step" in s
    assert "regresses kuma's client about 4×" in s and "0.57–0.71 GiB/s against 2.6–2.8 GiB/s" in s
    assert "supported only together with §3.3's `TxLoop`" in s
    r = norm(open(os.path.join(ROOT, "README.md")).read())
    assert "regresses kuma's client about 4×" in r and "supported only together with `TxLoop`" in r


def test_timeout_switch_off_and_thread_rules_documented():
    s = norm(section(open(os.path.join(ROOT, "INTEGRATION.md")).read(), "## 5. Threading"))
    assert "`KMWS_ERR_TIMEOUT` switches the grid off for the whole process" in s
    assert "for the rest of its life" in s
    assert "KMWS_DEVICE_AUTO" in s and "KMWS_DEVICE_POLICY_NUMA" in s
    assert "**Thread exit.**" in s and "kmws_thread_attach" in s


def test_design_resize_poll_matches_the_kernel():
    """DESIGN.md's account of the resize word matches kmws_resident.hip (every
    16th poll)."""
    src = open(os.path.join(ROOT, "kuma_amd", "csrc", "kmws_resident.hip")).read()
    assert "if ((it & 15u) == 0) resize = ld_sys(&mb->resize);" in src
    d = norm(open(os.path.join(ROOT, "DESIGN.md")).read())
    assert "every fourth poll" not in d
