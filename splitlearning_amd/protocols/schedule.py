"""The Bob-side schedule of each mode (reference `split_nn.py:34-146`), executed
SPMD by every process.  Stdout lines are the reference's; per-phase wall time and
samples/s are logged as "[perf]" lines and written to `<log_dir>/metrics.json`.

The schedule is a list of top-level steps (one reference call each, e.g.
`train_request(c)` of one iteration, `eval_request_breakdown`, `unlearn_request`).
With `--ckpt_dir` every rank snapshots its state after each step
(`runtime/snapshot.py`); `--resume` skips the steps a previous, interrupted run
completed and continues from there.
"""
from __future__ import annotations

from .base import Session


def _print(sess: Session, msg: str):
    if sess.rank == 0 and not getattr(sess, "quiet", False):
        print(msg, flush=True)


def build_steps(sess: Session, args) -> list:
    """[(name, fn)] in schedule order."""
    omit = args.omit_label
    unl = list(args.unlearn_client_ids)
    k = sess.k
    T = sess.timer
    mode = sess.mode
    ntr = sum(sess.n_train.values())
    nte = sum(sess.n_test.values())
    steps = []

    def add(name, fn):
        steps.append((name, fn))

    def eval_breakdown():
        with T.phase("eval_breakdown", nte):
            sess.eval_request_breakdown(omit)

    def server(phase, ids, uid):
        def fn():
            with T.phase(phase) as box:
                box["samples"] = _agree(sess, sess.train_and_backward(ids, uid))
        return fn

    if mode in ("vanilla", "ushape"):
        for it in range(args.iterations):
            for cid in range(1, k + 1):
                def train(cid=cid):
                    _print(sess, f"Training client {cid}")
                    with T.phase(f"train_request[{cid}]", sess.n_train[cid] * args.epochs):
                        sess.train_request(cid)
                add(f"iter{it}.train_request[{cid}]", train)
            add(f"iter{it}.eval_breakdown", eval_breakdown)
        for it in range(args.iterations):
            def unlearn():
                with T.phase(f"unlearn_request[{unl[0]}]") as box:
                    sess.unlearn_request(unl[0], omit)
                    box["samples"] = sess.unlearn_samples(unl[0]) * args.epochs
            add(f"unlearn{it}.unlearn_request[{unl[0]}]", unlearn)
            add(f"unlearn{it}.eval_breakdown", eval_breakdown)

    elif mode in ("concat", "sisa"):
        def local():
            _print(sess, "Training all clients in parallel")
            with T.phase("local_training", ntr * args.epochs):
                sess.train_request_parallel()
            sess.freeze_alice_weights(range(1, k + 1))
            _print(sess, "Training server")
        add("local_training", local)
        add("server_training", server("server_training", [], None))
        add("eval_breakdown", eval_breakdown)
        if mode == "sisa" or args.concat_unlearn:
            def unlearn_local():
                sess.unfreeze_alice_weights(unl)
                _print(sess, f"Retraining client {unl}")
                with T.phase("unlearn_local") as box:
                    sess.unlearn_request(unl[0], omit)
                    box["samples"] = sess.unlearn_samples(unl[0]) * args.epochs
                sess.freeze_alice_weights(unl)
                _print(sess, "Retraining server upon the omitted labels")
            add("unlearn_local", unlearn_local)
            add("server_retraining", server("server_retraining", unl, omit))
            add("eval_breakdown_after", eval_breakdown)

    elif mode == "control":
        for it in range(args.iterations):
            for cid in range(1, k + 1):
                def local(cid=cid):
                    _print(sess, f"(Control group) Training client {cid}")
                    with T.phase(f"control_local[{cid}]"):
                        if cid in unl:
                            sess.train_request_control(cid, omit)
                        else:
                            sess.train_request(cid)
                add(f"iter{it}.control_local[{cid}]", local)
        add("freeze", lambda: sess.freeze_alice_weights(range(1, k + 1)))
        for it in range(args.iterations):
            def srv():
                _print(sess, "(Control group) Training server")
                server("server_training", unl, omit)()
                with T.phase("eval", nte):
                    sess.eval_request()
            add(f"iter{it}.server_training", srv)
    else:
        raise ValueError(mode)
    return steps


def run_schedule(sess: Session, args) -> dict:
    steps = build_steps(sess, args)
    ckpt = getattr(args, "ckpt_dir", "")
    start = 0
    if ckpt:
        from ..runtime import snapshot
        if getattr(args, "resume", False):
            start = snapshot.load(sess, ckpt)
            if start:
                sess.bob_log.info(f"[resume] {start} of {len(steps)} schedule steps completed; "
                                  f"continuing at {steps[start][0] if start < len(steps) else 'the end'}")
                _print(sess, f"Resuming after step {start}/{len(steps)}")
    for i, (name, fn) in enumerate(steps):
        if i < start:
            continue
        fn()
        if ckpt:
            snapshot.save(sess, ckpt, i + 1, name, getattr(args, "ckpt_keep", 2))
    return {"phases": sess.timer.records, "steps": [n for n, _ in steps], "resumed_at": start}


def _agree(sess: Session, n: int) -> int:
    """Sample counts are computed on Bob ranks; make rank 0's number authoritative."""
    return int(sess.comm.broadcast_obj(n, sess.pl.bob_root)) if sess.comm.distributed else n
