"""Load tests/golden/*.npz fixtures (numpy, allow_pickle=False) into VoteBatch + descriptors."""
import glob
import os

import numpy as np

from hashgraph_like_consensus import _ffi
from hashgraph_like_consensus.batch import VoteBatch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    batch = VoteBatch(vote_id=z["vote_id"], proposal_id=z["proposal_id"], timestamp=z["timestamp"], vote=z["vote"],
                      arena=z["arena"], field_off=z["field_off"], field_len=z["field_len"])
    desc = np.ascontiguousarray(z["desc"]).reshape(-1).view(_ffi.PROPOSAL_DTYPE)
    exp = dict(results=np.ascontiguousarray(z["exp_results"]).reshape(-1).view(_ffi.RESULT_DTYPE),
               vote_status=z["exp_vote_status"], vote_reason=z["exp_vote_reason"], recovered=z["exp_recovered"])
    return batch, desc, int(z["now"]), exp
