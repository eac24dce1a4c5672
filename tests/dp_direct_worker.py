"""One rank of tests/test_update_parity.py::test_direct_path_data_parallel_matches_hand_averaged_reference_gpu,
launched by torch.distributed.run (2 ranks, gloo, VSS_LOCAL_DEVICE=0): ppo_update over this rank's batch the
way train() sets it up -- FlatGrads with flat parameters, FlatAdam, the captured direct minibatch, --norm-adv
with the advantage statistics of both ranks' rows -- then the weights into <out>/w<rank>.pt."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (HERE, os.path.join(REPO, "rsoccer-isaac-cleanrl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from vss_amd.minibatch import disable_graph_packet_capture  # noqa: E402

disable_graph_packet_capture()  # before anything initialises the GPU

import torch  # noqa: E402

import ppo_continuous_action_isaacgym as P  # noqa: E402
from test_ppo import _args, make_agent  # noqa: E402
from test_update_parity import COEF, DP_EPOCHS, DP_N, dp_rank_batch  # noqa: E402


def main(out_dir: str):
    world, rank, local = P.setup_distributed()
    assert world == 2
    device = torch.device(f"cuda:{local}")
    obs, act, logp, adv, ret, val = [t.to(device) for t in dp_rank_batch(rank)]
    agent = make_agent(2).to(device)
    flat = P.FlatGrads(agent, flat_params=True)
    opt = P.FlatAdam(flat, lr=1e-3, eps=1e-5)
    args = _args(norm_adv=True, global_adv_norm=True, num_minibatches=2, update_epochs=DP_EPOCHS, max_grad_norm=1.5,
                 **COEF)
    graph = P.make_minibatch_graph(agent, flat, args, DP_N, (52,), (2,), device)
    gen = torch.Generator(device=device).manual_seed(7 + rank)
    P.ppo_update(agent, opt, flat, args, obs, logp, act, adv, ret, val, world=world, gen=gen, graph=graph)
    torch.cuda.synchronize()
    w = torch.cat([p.detach().reshape(-1) for p in agent.parameters()]).cpu()
    torch.save(w, os.path.join(out_dir, f"w{rank}.pt"))
    with open(os.path.join(out_dir, f"info{rank}.txt"), "w") as f:
        f.write(f"direct={int(graph is not None and graph.direct)} graph={int(graph is not None and graph.graph is not None)} "
                f"replays={graph.replays if graph is not None else 0}\n")
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
