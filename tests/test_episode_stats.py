"""vss_episode_stats vs the reference's RecordEpisodeStatisticsTorch.step
(envs/wrappers.py:66-87) restated in torch: running returns / lengths and the returned copies
bit-exact; the 'return' entry (the reference's r.sum(1)) equals ((r0 + r1) + r2) + r3 bit for bit
and torch's sum within 1 ulp-scale tolerance."""
import pytest
import torch

from vss_amd import _native as N

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def reference_step(ep_ret, ep_len, rews, dones):
    ep_ret += rews
    ep_len += 1
    ret, ln = ep_ret.clone(), ep_len.clone()
    ep_ret *= 1 - dones.unsqueeze(1)
    ep_len *= 1 - dones
    return ret, ln, ret.sum(1)


@pytest.mark.parametrize("rows", [1, 255, 65536 + 7])
def test_episode_stats_kernel_matches_reference(rows):
    g = torch.Generator(device=DEV).manual_seed(rows)
    ep_ret = torch.zeros((rows, 4), device=DEV)
    ep_len = torch.zeros(rows, dtype=torch.int32, device=DEV)
    ref_ret, ref_len = ep_ret.clone(), ep_len.clone()
    out_ret = torch.empty_like(ep_ret)
    out_len = torch.empty_like(ep_len)
    out_sum = torch.empty(rows, device=DEV)
    lib = N.load()
    for t in range(40):
        rews = torch.randn((rows, 4), device=DEV, generator=g) * 3
        dones = (torch.rand(rows, device=DEV, generator=g) < 0.1).long()
        rc = lib.vss_episode_stats(N.stream_of(torch.device(DEV)), rows, rews.data_ptr(), dones.data_ptr(),
                                   ep_ret.data_ptr(), ep_len.data_ptr(), out_ret.data_ptr(), out_len.data_ptr(),
                                   out_sum.data_ptr())
        assert rc == 0
        want_ret, want_len, want_sum = reference_step(ref_ret, ref_len, rews, dones)
        assert torch.equal(out_ret.view(torch.int32), want_ret.view(torch.int32)), t   # incl. -0.0
        assert torch.equal(out_len, want_len)
        assert torch.equal(ep_ret.view(torch.int32), ref_ret.view(torch.int32))
        assert torch.equal(ep_len, ref_len)
        seq = ((want_ret[:, 0] + want_ret[:, 1]) + want_ret[:, 2]) + want_ret[:, 3]
        assert torch.equal(out_sum, seq)
        torch.testing.assert_close(out_sum, want_sum, rtol=1e-6, atol=1e-5)
    if rows > 100:  # sequences long enough to cover both: running episodes and fresh resets
        assert int(ep_len.max()) > 5 and int((ep_len == 0).sum()) > 0


def test_wrapper_uses_the_kernel_and_reports_reference_keys():
    from envs.vss import VSS, default_cfg
    from envs.wrappers import RecordEpisodeStatisticsTorch, SingleAgent
    cfg = default_cfg(512)
    cfg["env"]["maxEpisodeLength"] = 5
    env = RecordEpisodeStatisticsTorch(SingleAgent(VSS(cfg, DEV, DEV, 0, True, False, False)), DEV)
    env.reset()
    total = torch.zeros(512, 4, device=DEV)
    for t in range(7):
        _, _, dones, info = env.step(torch.zeros((512, 2), device=DEV))
        assert set(info["r"]) == {"goal", "grad", "move", "energy", "return"}
        if t < 4:
            total += info["rews"]
    # every field times out at step 5 (index 4): returned length 5 and returned return = sum so far
    assert t == 6 and int(info["l"].max()) <= 5
