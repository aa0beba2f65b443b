"""RCCL channel (CU) budget (parallel/comm.py rccl_channel_budget): the measured 16-channel default
(profiles/r4_commload) is exported as NCCL_MAX_NCHANNELS, an explicit NCCL_MAX_NCHANNELS wins, 0
leaves RCCL its own choice, and the streaming data-gradient grid is sized to the CUs left (a
conservative 32 channels when RCCL's count is unknown; DLMPI_DGS_BLOCKS overrides)."""
from deeplearning_mpi_amd.parallel.comm import DEFAULT_RCCL_CHANNELS, rccl_channel_budget


def _clean(monkeypatch):
    for k in ("DLMPI_RCCL_CHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_MIN_NCHANNELS", "DLMPI_DGS_BLOCKS"):
        monkeypatch.delenv(k, raising=False)


def test_default_budget(monkeypatch):
    _clean(monkeypatch)
    b = rccl_channel_budget()
    assert DEFAULT_RCCL_CHANNELS == 16
    assert b["NCCL_MAX_NCHANNELS"] == "16" and b["dgrad_stream_blocks"] == 256 - 16


def test_explicit_nccl_env_wins(monkeypatch):
    _clean(monkeypatch)
    monkeypatch.setenv("NCCL_MAX_NCHANNELS", "8")
    monkeypatch.setenv("DLMPI_RCCL_CHANNELS", "32")
    b = rccl_channel_budget()
    assert b["NCCL_MAX_NCHANNELS"] == "8" and b["dgrad_stream_blocks"] == 248


def test_rccl_own_choice_sizes_the_grid_conservatively(monkeypatch):
    _clean(monkeypatch)
    monkeypatch.setenv("DLMPI_RCCL_CHANNELS", "0")
    b = rccl_channel_budget()
    assert b["NCCL_MAX_NCHANNELS"] is None and b["dgrad_stream_blocks"] == 256 - 32


def test_grid_override(monkeypatch):
    _clean(monkeypatch)
    monkeypatch.setenv("DLMPI_DGS_BLOCKS", "200")
    assert rccl_channel_budget()["dgrad_stream_blocks"] == 200


def test_destroying_one_communicator_keeps_the_other_ones_budget(monkeypatch):
    """with two RCCL communicators alive (bench --rccl1 builds one beside
    init_distributed's), destroying one must leave the streaming data-gradient grid sized for the
    other's channels; the default grid comes back only when none is left."""
    _clean(monkeypatch)
    from deeplearning_mpi_amd._ext import native
    from deeplearning_mpi_amd.parallel.bootstrap import LaunchInfo
    from deeplearning_mpi_amd.parallel.comm import RcclCommunicator

    class FakeNative:   # the raw communicator: only destroy() is used here
        def destroy(self):
            pass

    info = LaunchInfo("single", 0, 1, 0, 1)
    C = native()
    a = RcclCommunicator(info, "cpu", FakeNative(), budget={"dgrad_stream_blocks": 240})
    assert C.dgs_blocks() == 240
    b = RcclCommunicator(info, "cpu", FakeNative(), budget={"dgrad_stream_blocks": 224})
    assert C.dgs_blocks() == 224   # room for the channels of both
    b.destroy()
    assert C.dgs_blocks() == 240   # a's channels still hold their CUs
    b.destroy()                    # idempotent
    assert C.dgs_blocks() == 240
    a.destroy()
    assert C.dgs_blocks() == 256   # none left: the default grid


def test_dropped_communicator_releases_its_budget(monkeypatch):
    """a communicator dropped without destroy() must not hold its CUs for the rest of the
    process -- the live set is weak and collection recomputes the grid."""
    import gc

    _clean(monkeypatch)
    from deeplearning_mpi_amd._ext import native
    from deeplearning_mpi_amd.parallel.bootstrap import LaunchInfo
    from deeplearning_mpi_amd.parallel.comm import RcclCommunicator

    class FakeNative:
        def destroy(self):
            pass

    info = LaunchInfo("single", 0, 1, 0, 1)
    C = native()
    gc.collect()
    C.set_dgs_blocks(0)
    default = C.dgs_blocks()   # the grid with no communicator alive
    a = RcclCommunicator(info, "cpu", FakeNative(), budget={"dgrad_stream_blocks": 232})
    assert C.dgs_blocks() == 232
    del a
    gc.collect()
    assert C.dgs_blocks() == default
