"""hum_pack_rows (the learner feed's packing launch, include/humanoid_env.h) through parallel.TrajectoryGather on the
device: time-major step outputs [k, n, ...] of every dtype the bench gathers land in the lane-major fragment bit for
bit, including a partial fragment and uneven launch sizes; bad descriptors are refused."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.parallel import TrajectoryGather  # noqa: E402


@pytest.mark.parametrize("n", [4096, 37])
def test_pack_rows_fragments_equal_torch_transpose(n):
    dev = torch.device("cuda", 0)
    G = 32
    fields = [("obs", (70,), torch.float32), ("act", (17,), torch.float32), ("reward", (), torch.float32),
              ("done", (), torch.uint8), ("frame", (), torch.int32)]
    tg = TrajectoryGather(fields, [n], G, dev)
    g = torch.Generator(device=dev).manual_seed(3)
    ref = {"obs": [], "act": [], "reward": [], "done": [], "frame": []}
    t = 0
    for kk in (8, 16, 8, 5):   # 37 steps: fragment [0, 32) and a partial one [32, 37)
        out = {"obs": torch.rand(kk, n, 70, device=dev, generator=g), "act": torch.rand(kk, n, 17, device=dev, generator=g),
               "reward": torch.randn(kk, n, device=dev, generator=g),
               "done": (torch.rand(kk, n, device=dev, generator=g) < 0.3).to(torch.uint8),
               "frame": torch.randint(0, 1 << 30, (kk, n), device=dev, generator=g, dtype=torch.int32)}
        slot = (t // G) % 2
        tg.pack(slot, t % G, out)
        for f, x in out.items():
            ref[f].append(x.transpose(0, 1).cpu().numpy())
        t += kk
        if t % G == 0 or t == 37:
            tg.start(slot)
            tg.wait(slot)
            got = tg.result(slot)
            steps = G if t % G == 0 else t % G
            for f in ref:
                want = np.concatenate(ref[f], axis=1)
                assert got[f].shape[:2] == (n, G)
                np.testing.assert_array_equal(got[f][:, :steps].cpu().numpy(), want)
                ref[f] = []


def test_pack_rows_rejects_bad_descriptors():
    x = torch.zeros(4, 8, 3, device="cuda")
    f = N.HumPackField(src=x.data_ptr(), dst=x.data_ptr(), src_step=96, src_lane=12, dst_step=12, dst_lane=48,
                       row_bytes=6)   # neither one byte nor a multiple of 4
    arr = (N.HumPackField * 1)(f)
    assert N.lib().hum_pack_rows(arr, 1, 4, 8, 0, ctypes.c_void_p(0)) == N.HUM_ERR_ARG
    assert N.lib().hum_pack_rows(arr, 0, 4, 8, 0, ctypes.c_void_p(0)) == N.HUM_ERR_ARG


@pytest.mark.parametrize("dev_type", ["cuda", "cpu"])
def test_pack_refuses_a_launch_crossing_the_fragment(dev_type):
    """hum_pack_rows writes by offset and knows nothing of the fragment's capacity: TrajectoryGather.pack refuses
    t0 < 0, t0 + k > G and fields of different step counts before anything is written, on both paths."""
    dev = torch.device(dev_type, 0) if dev_type == "cuda" else torch.device("cpu")
    n, G = 16, 8
    tg = TrajectoryGather([("obs", (70,), torch.float32), ("done", (), torch.uint8)], [n], G, dev)
    before = tg.send[0].clone()
    mk = lambda k: {"obs": torch.ones(k, n, 70, device=dev), "done": torch.ones(k, n, dtype=torch.uint8, device=dev)}
    for t0, k in ((4, 5), (8, 1), (-1, 2)):
        with pytest.raises(ValueError):
            tg.pack(0, t0, mk(k))
    with pytest.raises(ValueError):
        tg.pack(0, 0, {"obs": torch.ones(2, n, 70, device=dev), "done": torch.ones(3, n, dtype=torch.uint8, device=dev)})
    assert torch.equal(tg.send[0], before)
    tg.pack(0, 4, mk(4))   # exactly filling the fragment is fine
