"""Build newsrec_amd models with the golden fixtures' configuration and parameters."""
import torch

from newsrec_amd.manager import ManagerConfig as Cfg, build_model  # noqa: F401


def load_golden_params(model, g):
    """Copy the golden's regenerated parameters into the model by reference state_dict name."""
    sd = model.state_dict()
    with torch.no_grad():
        for n in g.names:
            assert n in sd, "missing %s" % n
            sd[n].copy_(torch.from_numpy(g.params[n]))
