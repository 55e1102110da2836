"""parallel/diag.py: the facts an N > 1 bench run records about its RCCL communicator,
parsed from RCCL's debug log (NCCL_DEBUG=INFO lines; synthetic text in RCCL's format), and
the placement checks that make a mis-launched scaling run fail loudly."""
import os

from sparknet_amd.parallel import diag

LOG = """\
host:1234:1234 [0] NCCL INFO RCCL version 2.22.3+hip6.4 HEAD:abc
host:1234:1240 [0] NCCL INFO Channel 00/16 :    0   1   2   3   4   5   6   7
host:1234:1240 [0] NCCL INFO Channel 15/16 :    0   7   6   5   4   3   2   1
host:1234:1240 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC comm 0x1 nRanks 08
host:1234:1240 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC comm 0x1 nRanks 08
host:1234:1240 [0] NCCL INFO Channel 02/0 : 0[0] -> 7[7] via SHM/direct/direct comm 0x1 nRanks 08
host:1234:1240 [0] NCCL INFO 16 coll channels, 16 collnet channels, 0 nvls channels, 16 p2p channels
"""


def test_parse_rccl_log():
    d = diag.parse_rccl_log(LOG)
    assert d["version"] == "2.22.3+hip6.4"
    assert d["channels"] == 16
    assert d["transports"] == {"P2P/IPC": 2, "SHM/direct": 1}
    assert d["lines"] == 7
    assert diag.parse_rccl_log("")["channels"] is None


def test_rccl_debug_env_and_read(tmp_path, monkeypatch):
    for k in ("NCCL_DEBUG", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS"):
        monkeypatch.delenv(k, raising=False)
    pat = diag.rccl_debug_env(str(tmp_path))
    assert os.environ["NCCL_DEBUG"] == "INFO" and os.environ["NCCL_DEBUG_FILE"] == pat
    (tmp_path / os.path.basename(pat.replace("%h", "hostA").replace("%p", "99"))).write_text(LOG)
    d = diag.read_rccl_logs(pat)
    assert d["files"] == 1 and d["channels"] == 16
    # a user-chosen debug destination is left alone
    assert diag.rccl_debug_env(str(tmp_path)) is None


class _Comm:
    def __init__(self, world, devs):
        self.world_size, self.devs = world, devs

    def allgather_int(self, v):
        return list(self.devs)


def test_check_placement():
    assert diag.check_placement(None, 1, False, 0, 0) is None
    assert "world 2" in diag.check_placement(_Comm(2, [0, 1]), 8, False, 0, 0)
    assert "LOCAL_RANK" in diag.check_placement(_Comm(2, [0, 1]), 2, False, 0, 1)
    assert "share devices" in diag.check_placement(_Comm(2, [0, 0]), 2, False, 0, 0)
    assert diag.check_placement(_Comm(2, [0, 0]), 2, True, 0, 1) is None  # --share-gpu rehearsal
