"""Command-line configuration, validation and protocol constants.

Flag names, types and defaults mirror the reference launcher
(`/root/reference/split_nn.py:152-166`) so an existing command line keeps
working; validation mirrors `split_nn.py:169-174`.  Constants the reference
hard-codes (`split_nn.py:27-28,44-45`, `models.py:50,52`,
`data_entities_vanilla_sisa.py:48,266`, `data_entities_vanilla.py:41`) become
configurable with the same defaults.  Everything below the "framework" banner
is new: device/placement, dtype, seeding and quirk switches.
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass

# Protocol constants (reference defaults).
DEFAULT_OMIT_LABEL = 9                 # split_nn.py:45
DEFAULT_UNLEARN_CLIENTS = (1,)         # split_nn.py:44
DROPOUT_P = 0.5                        # models.py:50,52
ADAM_WEIGHT_DECAY = 1e-5               # data_entities_vanilla_sisa.py:48,266
SGD_MOMENTUM = 0.9                     # data_entities_vanilla.py:41
TEST_PARTITION = 0.2                   # mnist_flat_generator.py:37
MIN_SAMPLES_PER_CLIENT = 10            # noniid_partition.py:44
CUT_FEATURES = 32 * 13 * 13            # models.py:35,49 (5408)
NUM_CLASSES = 10                       # MNIST


MODES = ("ushape", "vanilla", "sisa", "concat", "control")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Split Learning Initialization (MI355X-native)")
    # ---- reference flags (split_nn.py:153-166) ----
    p.add_argument("--world_size", type=int, default=3,
                   help="1 server (Bob) + (world_size - 1) clients (Alices)")
    p.add_argument("--epochs", type=int, default=1,
                   help="client epochs per train request (local epochs in SISA)")
    p.add_argument("--iterations", type=int, default=5,
                   help="round-robin rounds (ignored by SISA / concat, as in the reference)")
    p.add_argument("--batch_size", type=int, default=16)
    p.add_argument("--partition_alpha", type=float, default=0.5,
                   help="Dirichlet concentration for the non-IID partition")
    p.add_argument("--datapath", type=str, default="data/mnist_flat",
                   help="directory holding data_worker{k}_{train,test}.pt shards")
    p.add_argument("--lr", type=float, default=0.001)
    p.add_argument("--server_epochs", type=int, default=3,
                   help="Bob's server epochs (SISA)")
    p.add_argument("--vanilla", action="store_true", help="vanilla split-NN (labels to Bob)")
    p.add_argument("--sisa", action="store_true", help="SISA split learning + unlearning")
    p.add_argument("--concat", action="store_true", help="SISA with concatenated client embeddings")
    p.add_argument("--control", action="store_true", help="retrain-from-scratch control group")
    # ---- framework flags (new) ----
    g = p.add_argument_group("framework")
    g.add_argument("--device", choices=("auto", "cpu", "cuda"), default="auto",
                   help="auto = one process per visible GPU if any, else CPU processes")
    g.add_argument("--nprocs", type=int, default=0,
                   help="number of OS processes (0 = #GPUs on GPU, world_size on CPU)")
    g.add_argument("--bob_tp", type=int, default=0,
                   help="tensor-parallel degree of Bob's server tail (0 = all processes on GPU, 1 on CPU)")
    g.add_argument("--calibrate", action="store_true",
                   help="with --bob_tp 0 on several GPUs: measure the per-batch message cost over the "
                        "job's own links at start-up (parallel/calibrate.py) and pick Bob's TP degree "
                        "from it instead of the assumed MSG_US (or SL_MSG_US)")
    g.add_argument("--backend", choices=("auto", "nccl", "gloo"), default="auto")
    g.add_argument("--act_dtype", choices=("fp32", "bf16"), default="fp32",
                   help="wire dtype of every cut-layer activation transfer (per-batch vanilla / U-shape "
                        "messages, eval, SISA's dump and cache); compute stays fp32; bf16 halves the "
                        "traffic, rounding the activations")
    g.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32",
                   help="compute dtype of the GEMM-shaped ops (forward, data and weight gradients): "
                        "fp32 = exact fp32 MFMA (the reference's precision); bf16 = operands rounded to "
                        "bf16, fp32 accumulation (BASELINE config 2); master weights and optimizer "
                        "state stay fp32")
    g.add_argument("--kernels", choices=("auto", "hip", "torch"), default="auto",
                   help="compute path: hand-written HIP kernels (GPU) or torch ops")
    g.add_argument("--seed", type=int, default=None, help="seed everything (reference is unseeded)")
    g.add_argument("--num_samples", type=int, default=70000,
                   help="synthetic MNIST-shaped dataset size (no network: fetch_openml unavailable)")
    g.add_argument("--mnist_npz", type=str, default="",
                   help="optional local MNIST .npz (x uint8 [N,28,28], y [N]) used instead of synthetic")
    g.add_argument("--data_layout", choices=("image", "flat"), default="image",
                   help="shard rows as [1,28,28] images (load_mnist_image) or flat 784-vectors "
                        "(load_mnist_flat); the client front reads either")
    g.add_argument("--reuse_data", action="store_true",
                   help="reuse existing shards instead of regenerating (reference regenerates, Q12)")
    g.add_argument("--log_dir", type=str, default="logs")
    g.add_argument("--save_dir", type=str, default="",
                   help="write checkpoints (reference state_dict key names) at the end of the run")
    g.add_argument("--resume_dir", type=str, default="",
                   help="load checkpoints written by --save_dir before the schedule starts")
    g.add_argument("--ckpt_dir", type=str, default="",
                   help="write a full snapshot (weights, optimizer slots, step counters, RNG states, "
                        "SISA activation cache) after every schedule step, one file per rank")
    g.add_argument("--resume", action="store_true",
                   help="resume from the latest complete snapshot in --ckpt_dir: completed schedule "
                        "steps are skipped and the run continues exactly where it stopped")
    g.add_argument("--ckpt_keep", type=int, default=2, help="snapshots kept in --ckpt_dir")
    g.add_argument("--master_addr", type=str, default="127.0.0.1")
    g.add_argument("--master_port", type=int, default=5689)
    g.add_argument("--omit_label", type=int, default=DEFAULT_OMIT_LABEL)
    g.add_argument("--unlearn_clients", type=str, default="1",
                   help="comma-separated Alice ids that request unlearning")
    g.add_argument("--true_reset", action="store_true",
                   help="re-initialise the client front on unlearn (reference reset is a no-op, Q4)")
    g.add_argument("--eval_dropout_fix", action="store_true",
                   help="put Bob in eval mode for vanilla evaluation (reference keeps dropout on, Q7)")
    g.add_argument("--concat_unlearn", action="store_true",
                   help="extend the concat schedule with unlearning + retrain (BASELINE config 5)")
    g.add_argument("--timeout_s", type=float, default=1800.0,
                   help="bounded wait for every collective / control message")
    g.add_argument("--watchdog", choices=("abort", "report", "off"), default="abort",
                   help="failure detection over the rendezvous store: a dead peer or (with "
                        "--stall_after_s) a job-wide stall is reported and, with 'abort', ends the job")
    g.add_argument("--dead_after_s", type=float, default=60.0,
                   help="a peer with no heartbeat for this long is declared dead")
    g.add_argument("--stall_after_s", type=float, default=0.0,
                   help="report a stall when no rank passes a phase boundary for this long (0 = off)")
    g.add_argument("--watchdog_interval", type=float, default=1.0)
    g.add_argument("--fault_inject", type=str, default="",
                   help="RANK:PHASE[:crash|hang|silent] - make RANK fail at the phase beacon PHASE "
                        "(tests the failure paths)")
    g.add_argument("--python_epoch", dest="native_epoch", action="store_false",
                   help="issue Bob's eager server steps from Python instead of the native "
                        "executor (_C.ServerEpoch); numerics are identical")
    g.add_argument("--torch_p2p", dest="native_comm", action="store_false",
                   help="GPU: move data-plane messages with torch.distributed isend/irecv instead of "
                        "the native RCCL communicators (per-batch p2p on the compute stream, TP "
                        "all-reduce inside the server step)")
    g.add_argument("--resident", choices=("auto", "off"), default="auto",
                   help="SISA server epochs of a narrow Bob shard (fc1 <= 768 rows: TP >= 7) as ONE "
                        "persistent launch per client epoch with the shard's weights and Adam state "
                        "held on-chip (csrc/resident.hip); 'auto' uses it where it fits and, "
                        "tensor-parallel, after a cross-rank self-test passed; 'off' = the "
                        "launch-per-stage executor")
    g.add_argument("--hybrid", choices=("auto", "off"), default="auto",
                   help="SISA server epochs of a WIDE Bob shard (TP 1..4: fc1 up to 5120 rows) as ONE "
                        "persistent launch per client epoch with fc2 / fc3 and the biases on-chip and "
                        "fc1's weights / Adam state streamed through the launch (csrc/hybrid.hip); "
                        "'auto' uses it where it fits and, tensor-parallel, after a cross-rank "
                        "self-test passed; 'off' = the launch-per-stage executor")
    g.add_argument("--split_persist", choices=("auto", "off"), default="auto",
                   help="vanilla epochs of an Alice co-located with a one-shard Bob as ONE persistent "
                        "launch per epoch: her conv front and Bob's whole tail, fc2 / fc3 on-chip, "
                        "fc1 streamed (csrc/vanilla.hip); 'off' = the per-batch native executor")
    g.add_argument("--persistent_failsafe", choices=("on", "off"), default="on",
                   help="copy Bob's shard (weights, optimizer state) before each persistent server "
                        "epoch; if the launch fails mid-epoch on any Bob rank, restore it on every "
                        "rank and continue on the launch-per-stage executor (about 0.1 ms per client "
                        "epoch at TP = 1); 'off' = a failed launch ends the job")
    g.add_argument("--split_channel", choices=("auto", "ipc", "rccl"), default="auto",
                   help="vanilla / U-shape with the Alice remote from a one-shard Bob: the native "
                        "split epoch's per-batch link.  'auto' / 'ipc' = one-kernel messages over "
                        "peer-mapped HBM (csrc/ipc_p2p.h) when every rank sets it up and passes its "
                        "self-test ('auto' falls back to RCCL), 'rccl' = ncclSend / ncclRecv")
    g.add_argument("--tp_allreduce", choices=("auto", "rccl"), default="auto",
                   help="Bob's per-step TP all-reduce: 'auto' = one kernel over peer-mapped HBM "
                        "(csrc/ipc_ar.h) when every Bob rank sets it up and passes its self-test, "
                        "RCCL otherwise; 'rccl' = always RCCL")
    g.add_argument("--native_p2p_shim", action="store_true",
                   help="CPU tests: run the GPU data-plane code path (grouped p2p with RCCL ordering "
                        "semantics) over gloo (parallel/dist.py GlooP2PShim)")
    g.add_argument("--msg_log", action="store_true",
                   help="record every data-plane message (op, src, dst, bytes) of this rank in "
                        "<log_dir>/messages_rank<r>.json (tests pin the per-batch message sequence)")
    g.add_argument("--serial_alices", dest="multi_alice", action="store_false",
                   help="step co-located Alices' SISA local epochs one after another instead of "
                        "together (one launch per step for all of them); numerics are identical")
    g.add_argument("--trace_dir", type=str, default="",
                   help="write a Chrome-trace timeline per rank (phases, data-plane ops with bytes, "
                        "device time of server / local epochs) to DIR/trace_rank<r>.json")
    g.add_argument("--no_tqdm", action="store_true")
    g.add_argument("--graphs", choices=("auto", "on", "off"), default="auto",
                   help="capture Bob's fixed-shape server steps in HIP graphs (auto: single-GPU "
                        "tail only; on: also a tensor-parallel tail, all-reduce inside the graph)")
    return p


def validate(args: argparse.Namespace) -> argparse.Namespace:
    """Reference validation (`split_nn.py:169-174`) plus derived fields."""
    if args.concat and not args.sisa:
        raise ValueError("The --concat option can only be used with the --sisa option.")
    if args.vanilla and (args.sisa or args.concat):
        raise ValueError("The --vanilla option cannot be used with --sisa or --concat.")
    if args.control and (args.vanilla or args.sisa or args.concat):
        raise ValueError("The --control option cannot be used with any other options.")
    if args.world_size < 2:
        raise ValueError("--world_size must be >= 2 (one Bob and at least one Alice)")
    if args.batch_size < 1:
        raise ValueError("--batch_size must be >= 1")
    args.client_num_in_total = args.world_size - 1          # split_nn.py:176
    args.class_num = NUM_CLASSES
    args.mode = mode_of(args)
    ids = [int(s) for s in str(args.unlearn_clients).split(",") if s.strip()]
    for i in ids:
        if not 1 <= i <= args.client_num_in_total:
            raise ValueError(f"unlearn client {i} is not an Alice id in 1..{args.client_num_in_total}")
    args.unlearn_client_ids = ids
    if getattr(args, "resume", False) and not getattr(args, "ckpt_dir", ""):
        raise ValueError("--resume needs --ckpt_dir")
    return args


def mode_of(args) -> str:
    """Dispatch precedence of `split_nn.py:13-23`; --control gets SISA semantics (Q2)."""
    if args.vanilla:
        return "vanilla"
    if args.concat:
        return "concat"
    if args.sisa:
        return "sisa"
    if args.control:
        return "control"
    return "ushape"


def parse_args(argv=None) -> argparse.Namespace:
    return validate(build_parser().parse_args(argv))


@dataclass
class OptimCfg:
    """Hyper-parameters of one optimizer slot (fused kernels read these)."""
    kind: str            # "adam" | "sgd"
    lr: float
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    weight_decay: float = 0.0
    momentum: float = 0.0
