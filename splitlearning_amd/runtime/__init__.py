from .launcher import main, launch, resolve, worker
