"""Bidirectional PointConv scene-flow network (teacher) — drop-in for the reference's
models_bid_pointconv.PointConvBidirection (models_bid_pointconv.py:14-207).

Same submodules, attribute names (=> the same 438 state_dict keys), inputs and 8-tuple
output.  MI355X-first restructuring of the forward, with identical per-sample arithmetic:

  * pc1 and pc2 share every encoder module and every cost-volume direction, and none of
    those layers has batch statistics, so both clouds run as ONE batch of 2B through the
    encoder (conv, FPS, kNN, PointConvD) and the decoder's feature upsampling: half the
    launches, twice the work per launch (FPS: 2B workgroups instead of B);
  * only the pc1-side layers (cost volume refinement, scene-flow estimators whose train-mode
    BatchNorm sees pc1 only, warping) run at batch B.
"""

import torch
import torch.nn as nn

from pointconv_util import (PointConvD, PointWarping, UpsampleFlow, CrossLayerLight as CrossLayer,
                            SceneFlowEstimatorResidual, Conv1d)
from pointconv_util import index_points_gather as index_points, index_points_group, square_distance  # noqa: F401
from loss_functions import multiScaleLoss  # noqa: F401  (the reference defines it here too)
import kdpc_native
import wgrad
from pointnet2 import pointnet2_utils

# False runs the decoder's flow-dependent searches in line (the tests' reference)
COORD_FORK = True
_coord_streams = {}  # (device index, forking stream handle) -> side stream
# the fork shares the parameter-gradient stream (idle during the forward); False gives it a
# stream of its own (test seam: tests/test_gpu_graph.py captures both)
SHARED_SIDE_STREAM = True


class _CoordFork:
    """The decoder's flow-dependent coordinate work on a second stream.

    At levels 2..0 the cost volume's kNN (every point's nearest in the other cloud, pc2
    warped by the upsampled flow) depends on the coarser level's flow, so it cannot join the
    one-step-ahead coordinate plan; but it depends on coordinates only, while the main stream
    still has the level's feature upsampling (deconv) to run.  cross_neighbours() issues the
    search on the side stream as soon as the warped cloud exists; ready() makes the main
    stream wait for it right before the cost volume, and then queues on the side stream the
    inverted indices that the backward would otherwise build on its critical path (the cost
    volume's CSR with ranks, the warping blend's CSR); join() (end of the forward) makes the
    main stream wait for them.  Training forwards only.  Same kernels on the same inputs:
    bit-identical to the in-line searches
    (tests/test_gpu_kd.py::test_coordinate_fork_is_bit_identical)."""

    def __init__(self, device, enabled=True):
        self.cur = self.side = None
        # training forwards only (the KD step turns it off for its student: distill.py
        # _kd_student_streams)
        if enabled and COORD_FORK and device.type == "cuda" and torch.is_grad_enabled():
            self.cur = torch.cuda.current_stream(device)
            if SHARED_SIDE_STREAM:
                # the parameter-gradient stream: idle during the forward, and one stream
                # fewer against the 4 hardware queues of the process
                self.side = wgrad.side_stream(device)
            else:
                key = (device.index, self.cur.cuda_stream)
                self.side = _coord_streams.get(key)
                if self.side is None:
                    self.side = _coord_streams[key] = torch.cuda.Stream(device=device)

    def cross_neighbours(self, cross, xa, warp_idx):
        """Issue cross.neighbours(xa) on the side stream -> a handle for ready(), or None
        (forward_pair then searches in line)."""
        if self.side is None:
            return None
        xa = xa.detach()
        self.side.wait_stream(self.cur)
        xa.record_stream(self.side)
        with torch.cuda.stream(self.side):
            idx = cross.neighbours(xa)
        idx.record_stream(self.cur)  # allocated on the side stream, read on the main one
        return idx, xa.shape[1], warp_idx, cross.pos1.out_channels

    def ready(self, pending):
        """The main stream waits for the search; the inverted indices the backward will read
        are then built on the side stream, beside the cost volume."""
        if pending is None:
            return None
        idx, n, warp_idx, d = pending
        self.cur.wait_stream(self.side)
        if torch.is_grad_enabled():
            keep = []
            with torch.cuda.stream(self.side):
                c = kdpc_native.csr_rank_of(idx, n)  # what the cost volume's backward reads
                keep += [c.offsets, c.perm, c.rank]
                if warp_idx is not None:
                    warp_idx.record_stream(self.side)
                    c = kdpc_native.csr_of(warp_idx, n)
                    keep += [c.offsets, c.perm]
            for t in keep:
                t.record_stream(self.cur)
        return idx

    def join(self):
        if self.side is not None:
            self.cur.wait_stream(self.side)

scale = 1.0


class PointConvBidirection(nn.Module):
    def __init__(self, weightnet=16):
        super().__init__()
        flow_nei = 32
        feat_nei = 16
        self.scale = scale
        # l0: 8192
        self.level0 = Conv1d(3, 32)
        self.level0_1 = Conv1d(32, 32)
        self.cross0 = CrossLayer(flow_nei, 32 + 32, [32, 32], [32, 32])
        self.flow0 = SceneFlowEstimatorResidual(32 + 64, 32, weightnet=weightnet)
        self.level0_2 = Conv1d(32, 64)
        # l1: 2048
        self.level1 = PointConvD(2048, feat_nei, 64 + 3, 64, weightnet=weightnet)
        self.cross1 = CrossLayer(flow_nei, 64 + 32, [64, 64], [64, 64])
        self.flow1 = SceneFlowEstimatorResidual(64 + 64, 64, weightnet=weightnet)
        self.level1_0 = Conv1d(64, 64)
        self.level1_1 = Conv1d(64, 128)
        # l2: 512
        self.level2 = PointConvD(512, feat_nei, 128 + 3, 128, weightnet=weightnet)
        self.cross2 = CrossLayer(flow_nei, 128 + 64, [128, 128], [128, 128])
        self.flow2 = SceneFlowEstimatorResidual(128 + 64, 128, weightnet=weightnet)
        self.level2_0 = Conv1d(128, 128)
        self.level2_1 = Conv1d(128, 256)
        # l3: 256
        self.level3 = PointConvD(256, feat_nei, 256 + 3, 256, weightnet=weightnet)
        self.cross3 = CrossLayer(flow_nei, 256 + 64, [256, 256], [256, 256])
        self.flow3 = SceneFlowEstimatorResidual(256, 256, weightnet=weightnet)
        self.level3_0 = Conv1d(256, 256)
        self.level3_1 = Conv1d(256, 512)
        # l4: 64
        self.level4 = PointConvD(64, feat_nei, 512 + 3, 256, weightnet=weightnet)
        # deconv
        self.deconv4_3 = Conv1d(256, 64)
        self.deconv3_2 = Conv1d(256, 64)
        self.deconv2_1 = Conv1d(128, 32)
        self.deconv1_0 = Conv1d(64, 32)
        self.warping = PointWarping()
        self.upsample = UpsampleFlow()

    # ---------------------------------------------------------------------------------
    # Every tensor below is point-major, (batch, points, channels), contiguous: a 1x1 conv is
    # one GEMM over the points, a concatenation is along the last dim, and the HIP gathers
    # read whole rows.  Only the returned views are permuted to the reference's (B,C,N).
    def precompute_fps(self, xyz1, xyz2):
        """The encoder's whole FPS chain for a pair batch, (2B, S_l) int32 per level
        (levels 1-4).  It depends on the coordinates only, so a training loop can run it for
        the NEXT batch on a side stream while this batch's forward/backward runs
        (distill.FpsPrefetch), and a KD step can share it between teacher and student (same
        clouds, same deterministic FPS)."""
        x = torch.cat([xyz1, xyz2], 0)
        out = []
        for down in (self.level1, self.level2, self.level3, self.level4):
            idx = pointnet2_utils.furthest_point_sample(x, down.npoint)
            out.append(idx)
            x = index_points(x, idx)
        return out

    # the decoder's flow-dependent searches and their CSRs on a side stream (_CoordFork)
    coord_fork = True

    # kNN searches of the forward whose inputs are coordinates only (the clouds and their FPS
    # subsets): 13 of the 19 searches.  The flow-dependent ones (the warping 3-NN and the
    # levels-0..2 cost volumes, whose query cloud is the warped pc2) stay in the forward.
    PLAN_KNN = ("enc1", "enc2", "enc3", "enc4", "encup", "cross3", "up2", "up1", "up0",
                "est3", "est2", "est1", "est0")
    # the searches whose backward reads the CSR slot of every (row, neighbour) (PointConv and
    # cost-volume backward: csr_rank_of); the 3-NN blends only need offsets / perm (csr_of)
    # the estimators' self-kNN (K=9): their PointConv backward runs tiled
    # (kdpc_native.tile_plan_of: rows + tile plan + the CSR of the partial rows) and their
    # WeightNet backward reads offsets / perm
    _PLAN_TILED = (frozenset(("est3", "est2", "est1", "est0")) if kdpc_native.TILED_PC
                   else frozenset())
    _PLAN_RANKED = frozenset(("enc1", "enc2", "enc3", "enc4", "cross3",
                              "est3", "est2", "est1", "est0")) - _PLAN_TILED

    def precompute_plan(self, xyz1, xyz2, csr=True):
        """precompute_fps() plus every coordinate-only kNN search of the forward (PLAN_KNN)
        and, with csr=True, the inverted indices their backward reads (offsets, perm[, rank]),
        as one flat list of int32 tensors: [4 FPS] + [13 kNN] + [CSR tensors in PLAN_KNN
        order].  Like the FPS chain it can run for the NEXT batch on a side stream
        (distill.FpsPrefetch / GraphedStep's forked stream) and be shared by a KD teacher and
        student; forward(fps_idx=plan) then takes its searches and CSRs from it.  Same
        kernels on the same inputs as the forward's own searches: identical results."""
        B = xyz1.shape[0]
        x = torch.cat([xyz1, xyz2], 0)
        fps, pcs = [], [x]
        downs = (self.level1, self.level2, self.level3, self.level4)
        for down in downs:
            idx = pointnet2_utils.furthest_point_sample(x, down.npoint)
            fps.append(idx)
            x = index_points(x, idx)
            pcs.append(x)
        knn, nref, ctr = {}, {}, {}
        for lv, down in enumerate(downs, start=1):
            knn[f"enc{lv}"] = down.neighbours(pcs[lv - 1], pcs[lv])
            nref[f"enc{lv}"] = pcs[lv - 1].shape[1]
        knn["encup"], nref["encup"] = self.upsample.neighbours(pcs[3], pcs[4]), pcs[4].shape[1]
        knn["cross3"], nref["cross3"] = self.cross3.neighbours(pcs[3]), pcs[3].shape[1]
        for lv in (2, 1, 0):
            knn[f"up{lv}"] = self.upsample.neighbours(pcs[lv], pcs[lv + 1])
            nref[f"up{lv}"] = pcs[lv + 1].shape[1]
        for lv, est in ((3, self.flow3), (2, self.flow2), (1, self.flow1), (0, self.flow0)):
            knn[f"est{lv}"] = est.neighbours(pcs[lv][:B])
            nref[f"est{lv}"] = pcs[lv].shape[1]
            ctr[f"est{lv}"] = pcs[lv][:B]
        out = fps + [knn[k] for k in self.PLAN_KNN]
        if csr:
            for k in self.PLAN_KNN:
                c = (kdpc_native.csr_rank_of(knn[k], nref[k]) if k in self._PLAN_RANKED
                     else kdpc_native.csr_of(knn[k], nref[k]))
                out += [c.offsets, c.perm] + ([c.rank] if k in self._PLAN_RANKED else [])
                if k in self._PLAN_TILED:
                    out += kdpc_native.tile_plan_tensors(
                        kdpc_native.tile_plan_of(knn[k], ctr[k], nref[k]))
        return out

    def _unpack_plan(self, plan, npts):
        """(fps list | None, {PLAN_KNN key: idx}) from a precompute_fps() / precompute_plan()
        result; the CSR tensors of a full plan are attached to their index tensors (the
        backward's csr_of / csr_rank_of then find them instead of rebuilding)."""
        if plan is None:
            return None, {}
        plan = list(plan)
        if len(plan) == 4:
            return plan, {}
        nk = len(self.PLAN_KNN)
        knn = dict(zip(self.PLAN_KNN, plan[4:4 + nk]))
        rest = plan[4 + nk:]
        if rest:
            nref = {"encup": npts[4], "cross3": npts[3]}
            for lv in (1, 2, 3, 4):
                nref[f"enc{lv}"] = npts[lv - 1]
            for lv in (0, 1, 2):
                nref[f"up{lv}"] = npts[lv + 1]
            for lv in (0, 1, 2, 3):
                nref[f"est{lv}"] = npts[lv]
            i = 0
            for k in self.PLAN_KNN:
                ranked = k in self._PLAN_RANKED
                offsets, perm = rest[i], rest[i + 1]
                rank = rest[i + 2] if ranked else None
                i += 3 if ranked else 2
                kdpc_native.attach_csr(knn[k], nref[k], offsets, perm, rank)
                if k in self._PLAN_TILED:
                    kdpc_native.attach_tile_plan(knn[k], nref[k], *rest[i:i + 5])
                    i += 5
        return plan[:4], knn

    def _encode(self, pc, color, fps_idx=None, knn=None):
        """Shared encoder on the pair batch (2B).  Returns per-level xyz, features, fps idx.
        fps_idx: optional precompute_fps() result for this batch; knn: the plan's searches."""
        pre = fps_idx if fps_idx is not None else [None] * 4
        knn = knn or {}
        feat_l0 = self.level0_1.cl(self.level0.cl(color))
        feat_l0_1 = self.level0_2.cl(feat_l0)
        levels = [(self.level1, self.level1_0, self.level1_1),
                  (self.level2, self.level2_0, self.level2_1),
                  (self.level3, self.level3_0, self.level3_1)]
        pcs, feats, feats_out, fps = [pc], [feat_l0], [feat_l0_1], []
        x, f = pc, feat_l0_1
        for lv, (down, mix, widen) in enumerate(levels):
            x, f, idx = down.forward_cl(x, f, pre[lv], knn.get(f"enc{lv + 1}"))
            f = mix.cl(f)
            pcs.append(x)
            feats.append(f)
            fps.append(idx)
            f = widen.cl(f)
            feats_out.append(f)
        pc_l4, feat_l4, _ = self.level4.forward_cl(x, f, pre[3], knn.get("enc4"))
        feat_l4_3 = self.deconv4_3.cl(self.upsample.forward_cl(x, pc_l4, feat_l4,
                                                               knn.get("encup")))
        return pcs, feats, feats_out, fps, feat_l4_3

    def forward(self, xyz1, xyz2, color1, color2, fps_idx=None):
        """xyz*, color*: (B,N,3).  Returns (flows, fps_pc1_idxs, fps_pc2_idxs, pc1, pc2,
        feat1s, feat2s, crosses) exactly as the reference (models_bid_pointconv.py:198-207):
        flows/pcs/features as (B,C,N) (views of the point-major tensors).
        fps_idx: optional precompute_fps() or precompute_plan() result for these clouds."""
        B = xyz1.shape[0]
        pc = torch.cat([xyz1, xyz2], 0)
        color = torch.cat([color1, color2], 0)
        npts = [pc.shape[1]] + [d.npoint for d in (self.level1, self.level2, self.level3,
                                                    self.level4)]
        fps_idx, knn = self._unpack_plan(fps_idx, npts)
        pcs, feats, feats_out, fps, feat_l4_3 = self._encode(pc, color, fps_idx, knn)
        # pc1 / pc2 halves of a pair-batch tensor through ONE split per tensor: the backward
        # of a split is one concatenation, where two separate slices would each allocate and
        # zero a full-size gradient and copy into it, and then add the two
        halves = {}

        def _half(t, i):
            h = halves.get(id(t))
            if h is None:
                h = halves[id(t)] = (t, t.split(B))
            return h[1][i]
        one = lambda t: _half(t, 0)  # noqa: E731
        two = lambda t: _half(t, 1)  # noqa: E731

        # ---- level 3 (coarsest): no prior flow
        c_feat_l3 = torch.cat([feats[3], feat_l4_3], dim=-1)
        f1n, f2n, cross3 = self.cross3.forward_pair(pcs[3], c_feat_l3, knn.get("cross3"))
        feat_est, flow = self.flow3.forward_cl(one(pcs[3]), one(feats[3]), cross3,
                                               knn_idx=knn.get("est3"))
        flows, crosses, up_feats = [flow], [cross3], []

        decoders = [(2, self.cross2, self.flow2, self.deconv3_2),
                    (1, self.cross1, self.flow1, self.deconv2_1),
                    (0, self.cross0, self.flow0, self.deconv1_0)]
        fork = _CoordFork(pc.device, self.coord_fork)
        for lv, cross, flow_est, deconv in decoders:
            # one 3-NN search per level pair serves all three upsamplings (both clouds'
            # features, and pc1's flow and estimator features: its first B rows)
            up_idx = knn.get(f"up{lv}")
            if up_idx is None:
                up_idx = self.upsample.neighbours(pcs[lv], pcs[lv + 1])
            up_idx1 = kdpc_native.batch_prefix(up_idx, B)  # pc1 half, CSR shared with up_idx
            pc1_lv, pc2_lv = one(pcs[lv]), two(pcs[lv])
            sflow = flow if self.scale == 1.0 else self.scale * flow  # x1.0 is exact
            # the flow chain first: the cost volume's search can then run on the side
            # stream while the feature upsampling below runs here
            up_flow = self.upsample.forward_cl(pc1_lv, one(pcs[lv + 1]), sflow, up_idx1)
            pc2_warp, warp_idx = self.warping.forward_cl(pc1_lv, pc2_lv, up_flow, with_idx=True)
            xa = torch.cat([pc1_lv, pc2_warp], 0)
            pending = fork.cross_neighbours(cross, xa, warp_idx)
            f_up = deconv.cl(self.upsample.forward_cl(pcs[lv], pcs[lv + 1],
                                                      torch.cat([f1n, f2n], 0), up_idx))
            up_feats.append(f_up)
            c_feat = torch.cat([feats[lv], f_up], dim=-1)
            feat_up = self.upsample.forward_cl(pc1_lv, one(pcs[lv + 1]), feat_est, up_idx1)
            new_feat1 = torch.cat([one(feats[lv]), feat_up], dim=-1)
            f1n, f2n, cost = cross.forward_pair(xa, c_feat, fork.ready(pending))
            feat_est, flow = flow_est.forward_cl(pc1_lv, new_feat1, cost, up_flow,
                                                 knn_idx=knn.get(f"est{lv}"))
            flows.insert(0, flow)
            crosses.insert(0, cost)
        fork.join()

        cn = lambda t: t.permute(0, 2, 1)  # noqa: E731  point-major -> reference (B,C,N) view
        pc1 = [cn(one(p)) for p in pcs]
        pc2 = [cn(two(p)) for p in pcs]
        fps_pc1_idxs = [one(i) for i in fps]
        fps_pc2_idxs = [two(i) for i in fps]
        # feat{1,2}s = [l0_1, l1_2, l2_3, l3_4, l3_2, l2_1, l1_0] (reference :203-204)
        enc = feats_out[:4]
        feat1s = [cn(one(t)) for t in enc] + [cn(one(t)) for t in up_feats]
        feat2s = [cn(two(t)) for t in enc] + [cn(two(t)) for t in up_feats]
        return ([cn(f) for f in flows], fps_pc1_idxs, fps_pc2_idxs, pc1, pc2, feat1s, feat2s,
                [cn(c) for c in crosses])
