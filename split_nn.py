"""Split learning + SISA unlearning on MI355X — reference-compatible command line.

    python split_nn.py [--world_size 3] [--epochs 1] [--iterations 5] [--batch_size 16]
                       [--partition_alpha 0.5] [--datapath data/mnist_flat] [--lr 0.001]
                       [--server_epochs 3] [--vanilla | --sisa [--concat] | --control]

Same flags, defaults and validation as /root/reference/split_nn.py:152-176; framework
flags (device placement, TP degree, seeding, ...) are listed by --help.
"""
from splitlearning_amd.runtime.launcher import main

if __name__ == "__main__":
    main()
