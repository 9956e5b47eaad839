"""Evaluation slice of the reference's core/function.py on the HIP path.

``validate_batch`` is the body of the reference's validation loop
(function.py:555-644) for one batch of V views: forward, optional flip test (mirrored
input folded into the input pack, heatmaps brought back / shifted / averaged by one
posu_flip_back launch per view), weighted-MSE loss, PCK accuracy, and
``get_final_preds`` per view with the predictions interleaved view-minor
(``preds[k::nviews]``) exactly as the reference stores them.  Everything stays on the
device until the final copy of predictions and heatmaps.

With NETWORK.AGGRE the cross-view Aggregation runs too (models.multiview_pose_resnet),
TEST.FUSE_OUTPUT routes the outputs (``fuse_routing``), and the loss carries the
reference's AGGRE terms (function.py:597-609): the consistent loss between the raw and
aggregated heatmaps of the H36M samples (LOSS.USE_CONSISTENT_LOSS, plain mean MSE) and,
with DATASET.PSEUDO_LABEL_PATH, the weighted MSE of the routed outputs against the
pseudo-label targets times LOSS.MSE_LOSS_WEIGHT.

``validate`` keeps the reference signature (function.py:529-536) and its outputs: the
``heatmaps_locations_<subset>_<type>.h5`` file that run/test/test_triangulate.py reads
(keys heatmaps / locations / joint_names_order, u2a-selected joints) and
``dataset.evaluate``'s perf indicator.  Debug-image dumps and tensorboard are not part
of this build.
"""
import logging
import os
import time

import numpy as np
import torch

from core.evaluate import accuracy
from core.inference import get_final_preds
from posu import ops
from utils.transforms import flip_pair_order

logger = logging.getLogger(__name__)


def fuse_routing(raw_features, aggre_features, is_aggre, meta):
    """function.py:33-45: per sample, 3/5 aggregated + 2/5 raw for H36M samples, raw
    otherwise (one masked blend per view on the device)."""
    if not is_aggre:
        return raw_features
    output = []
    for r, a, m in zip(raw_features, aggre_features, meta):
        h36m = torch.tensor([s == 'h36m' for s in m['source']], device=a.device).view(-1, 1, 1, 1)
        output.append(torch.where(h36m, 3 / 5 * a + 2 / 5 * r, r))
    return output


def select_out_h36m(raw_features, aggre_features, meta):
    """function.py:47-61: per view, the raw and aggregated heatmaps of the H36M samples."""
    raw_h36m, agg_h36m = [], []
    for r, a, m in zip(raw_features, aggre_features, meta):
        idx = torch.tensor([s == 'h36m' for s in m['source']], dtype=torch.bool, device=r.device)
        raw_h36m.append(r[idx])
        agg_h36m.append(a[idx])
    return raw_h36m, agg_h36m


def _run_model(model, views, hflip):
    """model(views) -> (per-view heatmaps, aggregated heatmaps or []); the flip test's
    mirrored input is packed by the HIP input-pack kernel when the model is this build's."""
    base = getattr(model, 'module', model)          # DDP-wrapped or not
    resnet = getattr(base, 'resnet', None)
    if hflip and resnet is not None and hasattr(resnet, 'plan') and not resnet.training:
        plan = resnet.plan(views[0].device)
        hm, _, _ = plan.run(plan.pack_input(views, hflip=True), keep_features=False)
        raw = list(torch.split(hm, views[0].shape[0], dim=0))
        agg = base.aggre_layer(raw) if getattr(base, 'aggre_layer', None) is not None else []
        return raw, agg
    if hflip:
        views = [torch.flip(v, dims=[3]) for v in views]
    raw, agg, _, _ = model(views)
    return raw, agg


def validate_batch(config, model, input, target=None, weight=None, meta=None, flip_pairs=None,
                   criterion=None, criterion_dict=None):
    """One batch of the reference's validate loop.

    input: V x [N, 3, H, W] cuda f32; target / weight: V x [N, J, h, w] / [N, J, 1] (optional);
    meta: V dicts with 'center', 'scale' ([N, 2]).  Returns a dict with
    output (V x [N, J, h, w] cuda), preds ([V*N, J, 3] numpy, row k::V = view k), heatmaps
    ([V*N, J, h, w] numpy, same order), loss (float or None), acc / cnt (or None)."""
    device = input[0].device
    nviews = len(input)
    fuse = bool(config.NETWORK.AGGRE) and bool(getattr(config.TEST, 'FUSE_OUTPUT', False))
    with torch.no_grad():
        raw, agg = _run_model(model, input, False)
        output = fuse_routing(raw, agg, fuse, meta) if fuse else raw
        if config.TEST.FLIP_TEST:
            raw_f, agg_f = _run_model(model, input, True)
            flipped = fuse_routing(raw_f, agg_f, fuse, meta) if fuse else raw_f
            perm = torch.tensor(flip_pair_order(output[0].shape[1], flip_pairs or []), dtype=torch.int32,
                                device=device)
            output = [ops.flip_back(f, perm, hm=o, shift=bool(config.TEST.SHIFT_HEATMAP))
                      for o, f in zip(output, flipped)]
        res = {'output': output, 'loss': None, 'acc': None, 'cnt': None}
        if target is not None:
            target = [t.to(device) for t in target]
            criterion = criterion or (criterion_dict or {}).get('mse_weights')
            if criterion is not None and weight is not None:
                weight = [w.to(device) for w in weight]
                loss = 0
                for t, w, r in zip(target, weight, raw):   # on the raw outputs (function.py:589-595)
                    loss = loss + criterion(r, t, w)
                if config.NETWORK.AGGRE:                   # function.py:597-609
                    if getattr(config.LOSS, 'USE_CONSISTENT_LOSS', False):
                        raw_h36m, agg_h36m = select_out_h36m(raw, agg, meta)
                        assert len(raw_h36m[0]) == len(agg_h36m[0])
                        if len(raw_h36m[0]) != 0:
                            rh, ah = torch.cat(raw_h36m, dim=0), torch.cat(agg_h36m, dim=0)
                            # torch.nn.MSELoss(reduction='mean') = the joints MSE (a sum of
                            # per-joint means) / J, on the HIP reduction kernel
                            loss = loss + ops.joints_mse(rh.contiguous(), ah.contiguous(), None) / rh.shape[1]
                    if getattr(config.DATASET, 'PSEUDO_LABEL_PATH', ''):
                        for t, w, o in zip(target, weight, output):
                            loss = loss + criterion(o, t, w) * config.LOSS.MSE_LOSS_WEIGHT
                res['loss'] = float(loss)
            accs, cnts = [], []
            for o, t in zip(output, target):
                _, a, c, _ = accuracy(o, t)
                accs.append(a)
                cnts.append(c)
            res['acc'], res['cnt'] = float(np.mean(accs)), float(np.mean(cnts))
        n = input[0].shape[0]
        njoints, h, w = output[0].shape[1:]
        preds = torch.empty((nviews * n, njoints, 3), dtype=torch.float32, device=device)
        hms = torch.empty((nviews * n, njoints, h, w), dtype=torch.float32, device=device)
        for k, (o, m) in enumerate(zip(output, meta)):
            center = m['center'].numpy() if hasattr(m['center'], 'numpy') else np.asarray(m['center'])
            scale = m['scale'].numpy() if hasattr(m['scale'], 'numpy') else np.asarray(m['scale'])
            p, mv = get_final_preds(config, o, center, scale)
            preds[k::nviews, :, 0:2] = p
            preds[k::nviews, :, 2:3] = mv
            hms[k::nviews] = o
        res['preds'] = preds.cpu().numpy()
        res['heatmaps'] = hms.cpu().numpy()
    return res


def save_heatmaps_locations(file_name, all_heatmaps, all_preds, u):
    """The validate() output file (function.py:671-676) read by test_triangulate.py."""
    try:
        import h5py
    except ImportError as e:  # not installed in this image; the format needs it
        raise ImportError('writing %s needs h5py (the reference writes HDF5 here)' % file_name) from e
    with h5py.File(file_name, 'w') as f:
        f['heatmaps'] = all_heatmaps[:, u, :, :]
        f['locations'] = all_preds[:, u, :]
        f['joint_names_order'] = u


def validate(config, loader, dataset, model_dict, criterion_dict, output_dir, writer_dict, rank):
    """function.py:529-690 without debug images: returns dataset.evaluate's perf indicator."""
    device = torch.device('cuda', rank)
    for model in model_dict.values():
        model.eval()
    nsamples = len(dataset) * 4
    njoints = config.NETWORK.NUM_JOINTS
    height = int(config.NETWORK.HEATMAP_SIZE[0])
    width = int(config.NETWORK.HEATMAP_SIZE[1])
    all_preds = np.zeros((nsamples, njoints, 3), dtype=np.float32)
    all_heatmaps = np.zeros((nsamples, njoints, height, width), dtype=np.float32)
    idx = 0
    end = time.time()
    for i, (input, target, weight, meta) in enumerate(loader):
        input = [view.to(device, non_blocking=False) for view in input]
        r = validate_batch(config, model_dict['base_model'], input, target, weight, meta,
                           flip_pairs=getattr(dataset, 'flip_pairs', None), criterion_dict=criterion_dict)
        nimgs = r['preds'].shape[0]
        all_preds[idx:idx + nimgs] = r['preds']
        all_heatmaps[idx:idx + nimgs] = r['heatmaps']
        idx += nimgs
        if i % config.PRINT_FREQ == 0 and rank == 0:
            logger.info('Test: [%d/%d]\tTime %.3f\tLoss %s\tAccuracy %s', i, len(loader), time.time() - end,
                        r['loss'], r['acc'])
        end = time.time()
    perf_indicator = 1000
    if rank == 0:
        u2a = {k: v for k, v in dataset.u2a_mapping.items() if v != '*'}
        u = np.array([m[0] for m in sorted(u2a.items(), key=lambda x: x[0])])
        file_name = os.path.join(output_dir, 'heatmaps_locations_%s_%s.h5' % (dataset.subset, dataset.dataset_type))
        save_heatmaps_locations(file_name, all_heatmaps, all_preds, u)
        _, perf_indicator = dataset.evaluate(all_preds[:, u, :],
                                             output_dir if config.DEBUG.SAVE_ALL_PREDS else None)
    return perf_indicator
