from .dist import Placement, Comm, init_process, make_tp_group
