"""The Bob-side schedule of each mode (reference `split_nn.py:34-146`), executed
SPMD by every process.  Stdout lines are the reference's; per-phase wall time and
samples/s are logged as "[perf]" lines and written to `<log_dir>/metrics.json`.
"""
from __future__ import annotations

from .base import Session


def _print(sess: Session, msg: str):
    if sess.rank == 0:
        print(msg, flush=True)


def run_schedule(sess: Session, args) -> dict:
    omit = args.omit_label
    unl = list(args.unlearn_client_ids)
    k = sess.k
    T = sess.timer
    mode = sess.mode
    ntr = sum(sess.n_train.values())
    nte = sum(sess.n_test.values())

    if mode in ("vanilla", "ushape"):
        for _ in range(args.iterations):
            for cid in range(1, k + 1):
                _print(sess, f"Training client {cid}")
                with T.phase(f"train_request[{cid}]", sess.n_train[cid] * args.epochs):
                    sess.train_request(cid)
            with T.phase("eval_breakdown", nte):
                sess.eval_request_breakdown(omit)
        for _ in range(args.iterations):
            with T.phase(f"unlearn_request[{unl[0]}]") as box:
                sess.unlearn_request(unl[0], omit)
            with T.phase("eval_breakdown", nte):
                sess.eval_request_breakdown(omit)

    elif mode == "concat":
        _print(sess, "Training all clients in parallel")
        with T.phase("local_training", ntr * args.epochs):
            sess.train_request_parallel()
        sess.freeze_alice_weights(range(1, k + 1))
        _print(sess, "Training server")
        with T.phase("server_training") as box:
            box["samples"] = _agree(sess, sess.train_and_backward([], None))
        with T.phase("eval_breakdown", nte):
            sess.eval_request_breakdown(omit)
        if args.concat_unlearn:
            sess.unfreeze_alice_weights(unl)
            _print(sess, f"Retraining client {unl}")
            with T.phase("unlearn_local"):
                sess.unlearn_request(unl[0], omit)
            sess.freeze_alice_weights(unl)
            _print(sess, "Retraining server upon the omitted labels")
            with T.phase("server_retraining") as box:
                box["samples"] = _agree(sess, sess.train_and_backward(unl, omit))
            with T.phase("eval_breakdown", nte):
                sess.eval_request_breakdown(omit)

    elif mode == "sisa":
        _print(sess, "Training all clients in parallel")
        with T.phase("local_training", ntr * args.epochs):
            sess.train_request_parallel()
        sess.freeze_alice_weights(range(1, k + 1))
        _print(sess, "Training server")
        with T.phase("server_training") as box:
            box["samples"] = _agree(sess, sess.train_and_backward([], None))
        with T.phase("eval_breakdown", nte):
            sess.eval_request_breakdown(omit)
        sess.unfreeze_alice_weights(unl)
        _print(sess, f"Retraining client {unl}")
        with T.phase("unlearn_local"):
            sess.unlearn_request(unl[0], omit)
        sess.freeze_alice_weights(unl)
        _print(sess, "Retraining server upon the omitted labels")
        with T.phase("server_retraining") as box:
            box["samples"] = _agree(sess, sess.train_and_backward(unl, omit))
        with T.phase("eval_breakdown", nte):
            sess.eval_request_breakdown(omit)

    elif mode == "control":
        for _ in range(args.iterations):
            for cid in range(1, k + 1):
                _print(sess, f"(Control group) Training client {cid}")
                with T.phase(f"control_local[{cid}]"):
                    if cid in unl:
                        sess.train_request_control(cid, omit)
                    else:
                        sess.train_request(cid)
        sess.freeze_alice_weights(range(1, k + 1))
        for _ in range(args.iterations):
            _print(sess, "(Control group) Training server")
            with T.phase("server_training") as box:
                box["samples"] = _agree(sess, sess.train_and_backward(unl, omit))
            with T.phase("eval", nte):
                sess.eval_request()
    else:
        raise ValueError(mode)
    return {"phases": T.records}


def _agree(sess: Session, n: int) -> int:
    """Sample counts are computed on Bob ranks; make rank 0's number authoritative."""
    return int(sess.comm.broadcast_obj(n, sess.pl.bob_root)) if sess.comm.distributed else n
