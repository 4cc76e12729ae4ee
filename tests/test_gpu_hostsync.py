"""The step's host <-> device plumbing (recommenders/hip/hostsync.py): the
loss read-back and the inputs staged on a copy stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def test_input_stage_rotates_slots_and_keeps_every_step_its_own_inputs():
    """Ten puts of changing contents and shapes (pinned, pageable, numpy and
    device inputs, None): each step's device tensors equal that step's host
    inputs when a kernel on the launch stream reads them, even when the launch
    stream is kept busy so the copies of later steps run ahead of it."""
    import numpy as np

    from recommenders.hip.hostsync import InputStage
    st = InputStage(dev)
    big = torch.randn(2048, 2048, device=dev)
    seen = []
    for step in range(10):
        B = 64 if step < 6 else 32           # a short batch reallocates the slot's buffers
        s = (torch.arange(B * 5, dtype=torch.int64).view(B, 5) + 1000 * step)
        s = s.pin_memory() if step % 2 == 0 else s
        a = np.arange(B, dtype=np.int32) + step
        d = torch.full((B,), step, device=dev)
        big = big @ big.T / 2048             # keeps the launch stream busy
        out = st.put(s, a, d, None)
        assert out[2] is d and out[3] is None
        assert out[0].device.type == "cuda" and out[1].dtype == torch.int32
        seen.append((out[0].clone(), out[1].clone(), s.clone(), torch.as_tensor(a).clone()))
    torch.cuda.synchronize()
    for got_s, got_a, want_s, want_a in seen:
        assert torch.equal(got_s.cpu(), want_s) and torch.equal(got_a.cpu(), want_a)


def test_input_stage_disabled_copies_on_the_launch_stream(monkeypatch):
    from recommenders.hip.hostsync import InputStage
    monkeypatch.setattr(InputStage, "ENABLED", False)
    st = InputStage(dev)
    x = torch.arange(10)
    y, z = st.put(x, None)
    assert z is None and torch.equal(y.cpu(), x) and st.stream is None


def test_host_scalars_reads_the_captured_values():
    from recommenders.hip.hostsync import HostScalars
    h = HostScalars()
    for k in range(3):
        loss = torch.tensor([0.5 + k], device=dev)
        flag = torch.tensor([k], dtype=torch.int32, device=dev)
        h.capture(loss, flag)
        assert h.get() == [0.5 + k, float(k)]
