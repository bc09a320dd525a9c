"""Evaluation harness — the counterpart of the reference test.py (same flags,
same flow, same outputs), running AdaptedCLIP on the MI355X kernels.

    python test.py --dataset MVTec --img_size 336 --save_path ckpt/...     (needs weights + data)
    python test.py --dataset synthetic --allow_random_init --img_size 336  (C1: no files needed)
    python test.py --dataset synthetic_mvtec --allow_random_init --img_size 336  (C4's 15-class flow)
    torchrun --nproc-per-node 8 test.py ...   (C3-style: each class's images sharded over 8 GPUs)
    AACLIP_REHEARSAL=1 torchrun --nproc-per-node 2 test.py ...   (the same ranks, all on cuda:0 over gloo)

Differences from the reference, all on the host side:
  * the per-batch loop calls the fused AdaptedCLIP.predict (map + score in one
    device pass) and keeps results on the device (the reference syncs twice per
    batch, test.py:85,93); metrics_eval ranks the class's pixels on the device;
  * checkpoints load with torch.load(weights_only=True);
  * --allow_random_init / --dataset synthetic run without the OpenAI weights;
  * batch k+1 is copied to the device on a copy stream while batch k runs; masks
    stay on the device until metrics_eval;
  * under torchrun (WORLD_SIZE > 1, one process per GPU) every class's test set is
    sharded by image (aaclip.parallel.shard_range), each rank predicts its shard and
    the maps / scores / masks / labels are gathered (RCCL) onto rank 0, which runs
    metrics_eval and prints and logs the table.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
from glob import glob

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from dataset import DOMAINS, get_dataset  # noqa: E402
from forward_utils import get_adapted_text_embedding, metrics_eval_deferred, visualize  # noqa: E402
from model.adapter import AdaptedCLIP  # noqa: E402
from model.clip import create_model  # noqa: E402
from utils import setup_seed  # noqa: E402


def _device_batch(input_data, prep, device):
    """One loader batch -> (image fp32 [B,3,S,S], mask uint8 [B,1,S,S]) on the device:
    raw uint8 batches (dataset raw=True) go through aaclip_preprocess_images /
    aaclip_resize_masks_nearest, normalised ones are copied (non_blocking from the
    DataLoader's pinned memory). Runs on the caller's current stream."""
    if prep is not None:
        def run(fn, u8):
            if isinstance(u8, torch.Tensor):
                return fn(u8.to(device, non_blocking=True))
            return torch.cat([fn(t.to(device, non_blocking=True)[None]) for t in u8])
        image, mask = run(prep.images, input_data["image_u8"]), run(prep.masks, input_data["mask_u8"])
    else:
        image = input_data["image"].to(device, non_blocking=True)
        mask = torch.as_tensor(input_data["mask"]).to(device, non_blocking=True)
    return image, (mask != 0).to(torch.uint8)


def get_predictions(model, class_text_embeddings, test_loader, device, img_size, dataset="MVTec", prep=None,
                    n_total=None, streams=1):
    """test.py:53-99. Batch k+1 is copied to the device (and preprocessed, with prep) on a
    copy stream while batch k runs; maps, scores and masks stay on the device (the
    reference syncs twice per batch, test.py:85,93). Returns (masks uint8 [N,1,S,S]
    device tensor, labels numpy [N], maps [N,S,S] and scores [N] device tensors, file
    names). With n_total (sharded run: test_loader holds this rank's shard_range slice
    of a class's n_total images) the class is gathered in shard order onto rank 0, which
    alone runs metrics_eval; the other ranks return None for the tensors. A rank with an
    empty shard still takes part. streams: concurrent image chunks per batch (HIP
    streams) for batches of at least 8 images per chunk; results do not depend on it."""
    masks, labels, preds, preds_image, file_names = [], [], [], [], []
    device = torch.device(device)
    on_gpu = device.type == "cuda"  # (a CPU device only in the host-logic tests, with a stand-in model)
    main = torch.cuda.current_stream(device) if on_gpu else None
    copy = torch.cuda.Stream(device=device) if on_gpu else None

    def stage(batch):
        if not on_gpu:
            return (batch,) + _device_batch(batch, prep, device) + (None,)
        with torch.cuda.stream(copy):
            image, mask = _device_batch(batch, prep, device)
        ev = torch.cuda.Event()
        ev.record(copy)
        return batch, image, mask, ev

    it = iter(test_loader)
    first = next(it, None)
    staged = stage(first) if first is not None else None
    while staged is not None:
        input_data, image, mask, ready = staged
        if on_gpu:
            main.wait_event(ready)
            image.record_stream(main)
            mask.record_stream(main)
        class_name = input_data["class_name"]
        assert len(set(class_name)) == 1, "mixed class not supported"
        labels.append(np.asarray(input_data["label"]))
        file_names.extend(input_data["file_name"])
        nst = streams if image.shape[0] >= 8 * streams else 1
        pmap, score = model.predict(image, class_text_embeddings, DOMAINS[dataset], streams=nst)
        preds.append(pmap.clone())
        preds_image.append(score.clone())
        masks.append(mask)
        nxt = next(it, None)  # host: the next batch (loader workers) while this one runs
        staged = stage(nxt) if nxt is not None else None
    if preds:
        masks, labels = torch.cat(masks), np.concatenate(labels, axis=0)
        preds, preds_image = torch.cat(preds), torch.cat(preds_image)
    else:  # empty shard (fewer images than ranks): zero rows of the right shapes
        masks = torch.zeros(0, 1, img_size, img_size, device=device, dtype=torch.uint8)
        labels = np.zeros(0, dtype=np.int64)
        preds = torch.zeros(0, img_size, img_size, device=device)
        preds_image = torch.zeros(0, device=device)
    if n_total is not None:
        import torch.distributed as dist
        from aaclip.parallel import gather_rows_to
        lab = gather_rows_to(torch.from_numpy(labels.astype(np.int64)).to(device), n_total)
        masks, preds, preds_image = (gather_rows_to(t, n_total) for t in (masks, preds, preds_image))
        names = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
        dist.gather_object(file_names, names, dst=0)
        if dist.get_rank() != 0:
            return None, None, None, None, None
        labels = lab.cpu().numpy()
        file_names = [f for part in names for f in part]
    return masks, labels, preds, preds_image, file_names


def parse_args(argv=None):
    parser = argparse.ArgumentParser(description="Testing")
    parser.add_argument("--model_name", type=str, default="ViT-L-14-336", help="ViT-L-14-336")
    parser.add_argument("--img_size", type=int, default=518)
    parser.add_argument("--relu", action="store_true")
    parser.add_argument("--dataset", type=str, default="MVTec")
    parser.add_argument("--shot", type=int, default=4)
    parser.add_argument("--batch_size", type=int, default=32)
    parser.add_argument("--seed", type=int, default=111)
    parser.add_argument("--save_path", type=str, default="ckpt/baseline")
    parser.add_argument("--visualize", action="store_true")
    parser.add_argument("--text_norm_weight", type=float, default=0.1)
    parser.add_argument("--text_adapt_weight", type=float, default=0.1)
    parser.add_argument("--image_adapt_weight", type=float, default=0.1)
    parser.add_argument("--text_adapt_until", type=int, default=3)
    parser.add_argument("--image_adapt_until", type=int, default=6)
    # build-only flags
    parser.add_argument("--allow_random_init", action="store_true",
                        help="run on random-init CLIP + adapters when no checkpoints exist")
    parser.add_argument("--synthetic_n", type=int, default=16)
    parser.add_argument("--compute_dtype", type=str, default="fp16", choices=["bf16", "fp16", "fp32", "fp8"],
                        help="visual tower MFMA dtype: fp16 (default; meets the map-parity contract at the bf16 "
                             "rate), bf16, fp32 (fp32-MFMA parity mode) or fp8 (config C5)")
    parser.add_argument("--streams", type=int, default=2,
                        help="concurrent image chunks per batch on HIP streams (bit-identical results; "
                             "batches under 8 images per chunk run as one)")
    parser.add_argument("--gpu_preprocess", action=argparse.BooleanOptionalAction, default=True,
                        help="real datasets: decode on the host, resize + normalise on the GPU (bit-exact with the "
                             "Pillow path; the default); --no-gpu_preprocess = the Pillow transform in the workers")
    parser.add_argument("--results_json", type=str, default="",
                        help="also write the final table (rank 0) to this JSON file")
    return parser.parse_args(argv)


def main(argv=None):
    return run(parse_args(argv))[0]


def run(args):
    """main() body; returns (results DataFrame, context dict with the model, the text
    anchors and every class's (masks, labels, preds, preds_image)) for callers/tests."""
    setup_seed(args.seed)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if not torch.cuda.is_available():
        raise RuntimeError("the AA-CLIP MI355X build needs a GPU (no CPU path)")
    if world > 1:  # one process per GPU (torchrun); image-sharded classes
        import torch.distributed as dist
        # AACLIP_REHEARSAL=1: every rank on cuda:0 over gloo -- the multi-rank harness (shards,
        # gathers onto rank 0, rank-0 metrics) on a one-GPU box, where RCCL refuses two ranks
        # on one device (bench.py's AACLIP_BENCH_REHEARSAL is the same switch)
        rehearsal = os.environ.get("AACLIP_REHEARSAL") == "1"
        local = 0 if rehearsal else int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        if not dist.is_initialized():
            if rehearsal:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        device = torch.device("cuda", local)
    else:
        device = torch.device("cuda:0")
    os.makedirs(args.save_path, exist_ok=True)
    logger = logging.getLogger(__name__)
    if rank == 0:
        logging.basicConfig(filename=os.path.join(args.save_path, "test.log"), encoding="utf-8", level=logging.INFO)
    logger.info("args: %s", vars(args))

    clip_model = create_model(model_name=args.model_name, img_size=args.img_size, device=device,
                              pretrained=None if args.allow_random_init else "openai",
                              require_pretrained=not args.allow_random_init,
                              force_image_size=args.img_size if args.allow_random_init else None)
    clip_model.eval()
    model = AdaptedCLIP(clip_model=clip_model, text_adapt_weight=args.text_adapt_weight,
                        image_adapt_weight=args.image_adapt_weight, text_adapt_until=args.text_adapt_until,
                        image_adapt_until=args.image_adapt_until, relu=args.relu,
                        compute_dtype={"fp32": torch.float32, "fp8": torch.float8_e4m3fn, "fp16": torch.float16}.get(
                            args.compute_dtype, torch.bfloat16)).to(device)
    model.eval()

    text_file = glob(args.save_path + "/text_adapter.pth")
    if len(text_file) > 0:
        checkpoint = torch.load(text_file[0], map_location="cpu", weights_only=True)
        model.text_adapter.load_state_dict(checkpoint["text_adapter"])
        adapt_text = True
    else:
        adapt_text = False

    files = sorted(glob(args.save_path + "/image_adapter_*.pth"))
    if not files and args.allow_random_init:
        files = [None]
    assert len(files) > 0, "image adapter checkpoint not found"
    from pandas import DataFrame, Series
    for file in files:
        if file is not None:
            checkpoint = torch.load(file, map_location="cpu", weights_only=True)
            model.image_adapter.load_state_dict(checkpoint["image_adapter"])
            test_epoch = checkpoint["epoch"]
        else:
            test_epoch = -1
        logger.info("-----------------------------------------------")
        logger.info("load model from epoch %d", test_epoch)
        logger.info("-----------------------------------------------")
        synthetic = args.dataset.startswith("synthetic")
        raw = args.gpu_preprocess and not synthetic  # synthetic items are already normalised
        image_datasets = get_dataset(args.dataset, args.img_size, None, args.shot, "test", logger=logger,
                                     synthetic_n=args.synthetic_n, raw=raw)
        prep = None
        if raw:
            from aaclip.preprocess import Preprocessor
            prep = Preprocessor(args.img_size)
        with torch.no_grad():
            text_embeddings = get_adapted_text_embedding(model if adapt_text else clip_model, args.dataset, device)
        df = DataFrame(columns=["class name", "pixel AUC", "pixel AP", "image AUC", "image AP"])
        pending = []
        ctx = {"model": model, "text_embeddings": text_embeddings, "classes": {}}
        for class_name, image_dataset in image_datasets.items():
            workers = 0 if synthetic else 4
            from dataset import collate_raw
            n_total = None
            if world > 1:
                from aaclip.parallel import shard_range
                n_total = len(image_dataset)
                a, b = shard_range(n_total, rank, world)
                image_dataset = torch.utils.data.Subset(image_dataset, range(a, b))
            loader = torch.utils.data.DataLoader(image_dataset, batch_size=args.batch_size, shuffle=False,
                                                 num_workers=workers, pin_memory=True,
                                                 collate_fn=collate_raw if raw else None)
            with torch.no_grad():
                masks, labels, preds, preds_image, file_names = get_predictions(
                    model=model, class_text_embeddings=text_embeddings[class_name], test_loader=loader,
                    device=device, img_size=args.img_size, dataset=args.dataset, prep=prep, n_total=n_total,
                    streams=args.streams)
            if rank != 0:  # the class was gathered onto rank 0, which runs metrics_eval
                continue
            if args.visualize:
                visualize(masks.cpu().numpy(), preds.cpu().numpy(), file_names, args.save_path, args.dataset,
                          class_name=class_name)
            # enqueued now, read after the loop: the next class's batches start at once
            pending.append(metrics_eval_deferred(masks, labels, preds, preds_image, class_name,
                                                 domain=DOMAINS[args.dataset]))
            ctx["classes"][class_name] = (masks, labels, preds, preds_image)
        for read in pending:
            df.loc[len(df)] = Series(read())
        if rank != 0:
            continue
        df.loc[len(df)] = df.drop(columns=["class name"]).mean()
        df.loc[len(df) - 1, "class name"] = "Average"
        logger.info("final results:\n%s", df.to_string(index=False, justify="center"))
        print(df.to_string(index=False, justify="center"))
        if args.results_json:  # the table as JSON (tests compare sharded and single-process runs)
            import json
            with open(args.results_json, "w") as f:
                json.dump({"world": world, "rows": df.astype({c: float for c in df.columns[1:]}).to_dict("records")},
                          f)
    return df, ctx


if __name__ == "__main__":
    main()
