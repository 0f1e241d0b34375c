"""Batches of scene-flow samples staged into HBM one step ahead.

The reference iterates a torch DataLoader (pin_memory=True) and calls `.cuda()` on each of
the five tensors at the top of every step (distilTrain.py:160-166, evaluate_bid_pointconv.py
:109-118): the host-to-device copies then sit on the compute stream in front of the step.
DeviceLoader keeps the reference's DataLoader semantics (same collation into (B,N,3) float32
tensors, the same per-worker NumPy seeding so seeded runs draw the same samples) and issues
the copies of batch i+1 from pinned memory on a side HIP stream while batch i is being
consumed; the consumer's stream waits on an event, not on the host.  Each yielded tensor is
marked as used by the consumer stream (record_stream), so the caching allocator cannot
recycle it while the step still reads it."""
import numpy as np
import torch
import torch.utils.data as data


def collate_scene_flow(batch):
    """[(pc1, pc2, norm1, norm2, sf, path)] -> 5 stacked float32 tensors (B,N,3) + paths."""
    cols = list(zip(*batch))
    out = [torch.from_numpy(np.stack(c).astype(np.float32, copy=False)) for c in cols[:5]]
    return (*out, list(cols[5]))


def _seed_worker(worker_id):
    """The reference's worker_init_fn (distilTrain.py:73): NumPy's global generator seeded
    from torch's per-worker seed."""
    np.random.seed(torch.initial_seed() % (2 ** 32))


class DeviceLoader:
    """Iterable of (pos1, pos2, norm1, norm2, flow, paths) with the tensors on `device`."""

    def __init__(self, dataset, batch_size, device, shuffle=False, num_workers=0,
                 drop_last=False, generator=None):
        self.device = torch.device(device)
        self.on_gpu = self.device.type == "cuda"
        self.loader = data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle,
                                      num_workers=num_workers, pin_memory=self.on_gpu,
                                      collate_fn=collate_scene_flow, drop_last=drop_last,
                                      worker_init_fn=_seed_worker, generator=generator)
        self.stream = None

    def __len__(self):
        return len(self.loader)

    def _stage(self, batch):
        *tensors, paths = batch
        if not self.on_gpu:
            return tensors, paths, None
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=self.device)
        with torch.cuda.stream(self.stream):
            dev = [t.to(self.device, non_blocking=True) for t in tensors]
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return dev, paths, ev

    def __iter__(self):
        it = iter(self.loader)
        try:
            nxt = self._stage(next(it))
        except StopIteration:
            return
        while nxt is not None:
            tensors, paths, ev = nxt
            if ev is not None:
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                for t in tensors:
                    t.record_stream(cur)
            try:
                nxt = self._stage(next(it))
            except StopIteration:
                nxt = None
            yield (*tensors, paths)
