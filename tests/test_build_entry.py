"""__graft_entry__.build()'s rebuild rule: a library is rebuilt from scratch
when its sources' hash differs from the one recorded next to it, whatever
the files' timestamps say (a clock skew would otherwise ship a
stale library)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402


def test_rebuild_follows_the_source_hash_not_timestamps(tmp_path):
    src = tmp_path / "a.c"
    out = tmp_path / "out.txt"
    mk = tmp_path / "Makefile"
    src.write_text("one\n")
    mk.write_text("out.txt: a.c\n\tcat a.c >> out.txt\n")
    cmd = ["make", "-s", "-C", str(tmp_path)]
    ge._build_if_changed(str(out), [str(src), str(mk)], cmd)
    assert out.read_text() == "one\n"
    ge._build_if_changed(str(out), [str(src), str(mk)], cmd)      # unchanged: make is a no-op
    assert out.read_text() == "one\n"
    # the source changes but is made OLDER than the output (clock skew):
    # timestamps alone would keep the stale output; the hash forces make -B
    src.write_text("two\n")
    old = time.time() - 3600
    os.utime(src, (old, old))
    ge._build_if_changed(str(out), [str(src), str(mk)], cmd)
    assert out.read_text().endswith("two\n")
    assert (tmp_path / "out.txt.srchash").read_text().strip() == ge._sources_hash([str(src), str(mk)])


def test_product_stamp_matches_the_tree():
    """After build() the stamp next to the in-tree library is the current
    sources' hash (build() runs here if the library is missing or stale)."""
    csrc = os.path.join(ROOT, "etcd_amd", "csrc")
    prod = ge._listed(csrc, (".hip", ".cpp", ".h", ".py")) + [os.path.join(ROOT, "include",
                                                                          "quorum_batch.h")]
    stamp = os.path.join(ROOT, "etcd_amd", "libquorumbatch.so.srchash")
    if not os.path.exists(stamp) or open(stamp).read().strip() != ge._sources_hash(prod):
        ge.build()
    assert open(stamp).read().strip() == ge._sources_hash(prod)
