"""Reference-named role API over an SPMD session.

The reference exposes two classes per mode, `alice` and `bob`, whose methods Bob calls
over RPC (e.g. data_entities_vanilla_sisa.py:35-250 for `alice`,
:255-419 for `bob`).  Here a mode is one `Session` (protocols/) that every rank runs
in lock-step; `Bob` and `Alice` below are thin views that give the reference's method
names and signatures on top of it, so driver code written against the reference
(`bob.train_request(1)`, `alices[1].eval_breakdown(9)`, ...) ports line by line.

Every call is COLLECTIVE: all ranks of the job must make the same call in the same
order (it may move tensors between the Alice host rank and Bob's ranks).  Calls that
return per-client values return them on every rank.
"""
from __future__ import annotations

from .protocols.base import Session


class Alice:
    """View of client `cid` (reference `alice`, hosted on `session.host(cid)`)."""

    def __init__(self, session: Session, cid: int):
        self.s = session
        self.rank = cid

    # -- training ----------------------------------------------------------------
    def train(self, last_alice_rref=None, last_alice_id=None):
        """U/V: one sequential turn incl. the weight relay (data_entities_vanilla.py:56-76);
        SISA: local training (data_entities_vanilla_sisa.py:55-70)."""
        return self.s.train_request(self.rank)

    def train_control(self, omit_label: int):
        return self.s.train_control(self.rank, omit_label)

    def unlearn(self, omit_label: int):
        return self.s.unlearn_request(self.rank, omit_label)

    # -- weights -----------------------------------------------------------------
    def give_weights(self) -> dict | None:
        """state_dict of the client model(s) (on the host rank; None elsewhere)."""
        return self.s.give_weights(self.rank) if self.s.hosts(self.rank) else None

    def freeze_weights(self):
        self.s.freeze_alice_weights([self.rank])

    def unfreeze_weights(self):
        self.s.unfreeze_alice_weights([self.rank])

    def reset_model(self):
        if self.s.hosts(self.rank):
            self.s.reset_model(self.rank)

    # -- data / activations ------------------------------------------------------
    def load_data(self):
        """(train shard, test shard) device datasets (host rank; None elsewhere)."""
        a = self.s.alices.get(self.rank)
        return (a.train, a.test) if a is not None else None

    def give_activation_and_labels(self, unlearned: bool = False):
        """SISA: (acts [n,5408], labels [n]) as received by Bob (Bob ranks; None elsewhere)."""
        return self.s.get_activation_and_labels(self.rank, unlearned=unlearned,
                                                unlearn_id=getattr(self.s.args, "omit_label", None)
                                                if unlearned else None)

    # -- evaluation --------------------------------------------------------------
    def eval(self):
        """(correct, total) on this client's test shard."""
        self.s.before_eval()
        c = self.s._eval_counts(-1)
        return int(c[self.rank, 0]), int(c[self.rank, 1])

    def eval_breakdown(self, omit_label: int):
        """(corr, tot, corr_unlearned, tot_unlearned, corr_remaining, tot_remaining)."""
        self.s.before_eval()
        c = self.s._eval_counts(omit_label)
        return tuple(int(v) for v in c[self.rank])

    def start_logger(self):
        a = self.s.alices.get(self.rank)
        return a.logger if a is not None else None


class Bob:
    """Reference `bob`: the session's Bob-side API (train_request, eval_request, ...)
    plus `alices` (cid -> Alice view)."""

    def __init__(self, session: Session):
        self.s = session
        self.alices = {cid: Alice(session, cid) for cid in range(1, session.k + 1)}

    def __getattr__(self, name):
        # train_request, train_request_parallel, train_request_control, unlearn_request,
        # eval_request, eval_request_breakdown, freeze_alice_weights, unfreeze_alice_weights,
        # switch_mode_to_train/eval, train_and_backward, get_activation_and_labels, ...
        return getattr(self.s, name)

    def start_logger(self):
        return self.s.bob_log

    def inference(self, x):
        """Bob's forward on cut activations already on Bob's ranks (reference bob.inference)."""
        return self.s.inference(x)


def roles(session: Session) -> tuple[Bob, dict[int, Alice]]:
    bob = Bob(session)
    return bob, bob.alices
