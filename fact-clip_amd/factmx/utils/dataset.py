"""Dataset readers with the reference's names and outputs (fact_clip/utils/dataset.py):
``.npy`` frame features, ``groundTruth/<video>.txt`` per-frame label names,
``mapping.txt`` (``<index> <name>`` per line), split ``.bundle`` lists, the
holdout-class video filter and the batch iterator the training script drives.

On top of the reference surface, :class:`DevicePrefetcher` stages the next batch
into pinned host memory and copies it to the GPU on a side stream, so the H2D
copy of batch i+1 overlaps the fwd/bwd of batch i (the reference copies
synchronously inside the training loop, ``scripts/train.py``).

The data root defaults to ``$FACTMX_DATA_BASE`` or the repository root (the
reference uses the parent of its package, ``home.py:3-11``).
"""
import os

import numpy as np
import torch

from .utils import shrink_frame_label


def get_project_base():
    """home.py:3-11 analogue: ``$FACTMX_DATA_BASE`` or the directory above the package root."""
    env = os.environ.get("FACTMX_DATA_BASE")
    if env:
        return env.rstrip("/") + "/"
    pkg = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
    return os.path.dirname(pkg) + "/"


def load_feature(feature_dir, video, transpose):
    """dataset.py:12-21: ``<feature_dir>/<video>.npy`` as float32 (T, D); HAViD / Breakfast /
    GTEA store (D, T) and are transposed."""
    feature = np.load(os.path.join(feature_dir, video + ".npy"))
    if transpose:
        feature = feature.T
    if feature.dtype != np.float32:
        feature = feature.astype(np.float32)
    return feature


def load_action_mapping(map_fname, sep=" "):
    """dataset.py:23-35: ``mapping.txt`` -> (label2index, index2label); the name is everything
    after the first separator, the file's last line (after the final newline) is dropped."""
    label2index, index2label = {}, {}
    with open(map_fname, "r") as f:
        lines = f.read().split("\n")[:-1]
    for line in lines:
        idx, _, name = line.partition(sep)
        i = int(idx)
        label2index[name] = i
        index2label[i] = name
    return label2index, index2label


def _read_split(fname, strip_txt, txt_only):
    with open(fname, "r") as f:
        names = f.read().split("\n")[:-1]
    if txt_only:
        names = [v for v in names if v.endswith(".txt")]
    if strip_txt:
        names = [v[:-4] for v in names]
    return names


class Dataset:
    """dataset.py:37-77: lazy per-video cache of ``load_video_func(vname)`` ->
    (features (T, D) f32, training labels, evaluation labels)."""

    def __init__(self, video_list, nclasses, load_video_func, bg_class):
        self.video_list = video_list
        self.load_video = load_video_func
        self.nclasses = nclasses
        self.bg_class = bg_class
        self.data = {video_list[0]: load_video_func(video_list[0])}
        self.input_dimension = self.data[video_list[0]][0].shape[1]

    def __str__(self):
        return "< Dataset %d videos, %d feat-size, %d classes >" % (
            len(self.video_list), self.input_dimension, self.nclasses)

    __repr__ = __str__

    def get_vnames(self):
        return list(self.video_list)

    def __getitem__(self, video):
        if video not in self.video_list:
            raise ValueError(video)
        if video not in self.data:
            self.data[video] = self.load_video(video)
        return self.data[video]

    def __len__(self):
        return len(self.video_list)


class DataLoader:
    """dataset.py:80-131: batches of ``batch_size`` videos; the last batch wraps around to the
    start of the (shuffled) order; reshuffles (np.random) at the end of every epoch. Yields
    (video names, [float32 (T, D) tensors], [int64 (T,) tensors], [evaluation label lists]).

    Data parallel (factmx.dp): with ``world_size`` > 1 every rank walks the SAME global batch
    sequence (the shuffle comes from a RandomState seeded with ``seed``, identical on every rank,
    instead of the global np.random stream) and yields only its own share of each global batch,
    videos ``rank, rank + world_size, ...`` of it -- so the ranks' per-video losses together are
    exactly the reference's batch (blocks.py:913-915 averages them), and the DP all-reduce of the
    mean gradients equals the single-process gradient.  ``batch_size`` is the global batch and
    must be a multiple of ``world_size``."""

    def __init__(self, dataset, batch_size, shuffle=False, rank=0, world_size=1, seed=0):
        if world_size < 1 or not 0 <= rank < world_size:
            raise ValueError(f"rank {rank} / world_size {world_size}")
        if batch_size % world_size:
            raise ValueError(f"global batch {batch_size} is not a multiple of world_size {world_size}")
        self.num_video = len(dataset)
        self.dataset = dataset
        self.videos = list(dataset.get_vnames())
        self.shuffle = shuffle
        self.batch_size = batch_size
        self.rank, self.world_size = rank, world_size
        self._rng = np.random.RandomState(seed) if world_size > 1 else np.random
        self.num_batch = int(np.ceil(self.num_video / self.batch_size))
        self.selector = list(range(self.num_video))
        self.index = 0
        if self.shuffle:
            self._rng.shuffle(self.selector)

    def __len__(self):
        return self.num_batch

    def __iter__(self):
        return self

    def global_batch(self):
        """Video names of the next global batch (all ranks), advancing the iterator."""
        if self.index >= self.num_video:
            if self.shuffle:
                self._rng.shuffle(self.selector)
            self.index = 0
            raise StopIteration
        idx = self.selector[self.index:self.index + self.batch_size]
        if len(idx) < self.batch_size:
            idx = idx + self.selector[:self.batch_size - len(idx)]
        self.index += self.batch_size
        return [self.videos[i] for i in idx]

    def __next__(self):
        videos = self.global_batch()[self.rank::self.world_size]
        seqs, train_labels, eval_labels = [], [], []
        for v in videos:
            seq, tl, el = self.dataset[v]
            seqs.append(torch.from_numpy(seq))
            train_labels.append(torch.as_tensor(tl, dtype=torch.long))
            eval_labels.append(el)
        return videos, seqs, train_labels, eval_labels


class DevicePrefetcher:
    """Wraps a :class:`DataLoader`: batch i+1 is pinned and copied host->device on a dedicated
    stream while the caller computes on batch i. Yields the DataLoader's tuple with the sequence
    and label tensors on ``device``; the consumer stream waits on the copy's event, and each
    tensor is recorded on the consumer stream so the caching allocator cannot recycle it early."""

    def __init__(self, loader, device="cuda"):
        self.loader = loader
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(device=self.device)
        self._next = None

    def __len__(self):
        return len(self.loader)

    def _stage(self):
        try:
            names, seqs, labels, evals = next(self.loader)
        except StopIteration:
            self._next = None
            return
        with torch.cuda.stream(self.stream):
            dseq = [s.pin_memory().to(self.device, non_blocking=True) for s in seqs]
            dlab = [l.pin_memory().to(self.device, non_blocking=True) for l in labels]
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self._next = (names, dseq, dlab, evals, ev)

    def __iter__(self):
        self._stage()
        return self

    def __next__(self):
        if self._next is None:
            raise StopIteration
        names, dseq, dlab, evals, ev = self._next
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        for t in dseq + dlab:
            t.record_stream(cur)
        self._stage()
        return names, dseq, dlab, evals


def _read_gt_names(path):
    """Label-name lines of a groundTruth file: CRLF tolerated, utf-8 then latin-1 (dataset.py:150-156)."""
    with open(path, "rb") as f:
        raw = f.read().replace(b"\r\n", b"\n")
    try:
        text = raw.decode("utf-8")
    except UnicodeDecodeError:
        text = raw.decode("latin-1")
    return text.split("\n")[:-1]


def video_contains_holdout_classes(vname, groundTruth_path, label2index, holdout_classes):
    """dataset.py:137-167: does the video's ground truth contain any holdout class? Unreadable
    files count as "no" (with a warning), as in the reference."""
    try:
        names = _read_gt_names(os.path.join(groundTruth_path, vname + ".txt"))
        return any(label2index[n] in holdout_classes for n in names if n in label2index)
    except Exception as e:  # noqa: BLE001  (reference behaviour: warn and keep the video)
        print(f"Warning: Could not read labels for video {vname}: {e}")
        return False


# dataset.py:171-242, one row per dataset family: mapping / root / features / splits (relative
# to the data base), feature layout, background class ids, average transcript length.
def _dataset_spec(cfg, base):
    name = cfg.dataset
    o2o = cfg.Loss.match == "o2o"
    if name == "breakfast" or name == "gtea":
        root = f"{base}data/{name}/"
        return dict(mapping=root + "mapping.txt", root=root,
                    features=root + ("features" if name == "breakfast" else "features/"),
                    train=root + f"splits/train.{cfg.split}.bundle", test=root + f"splits/test.{cfg.split}.bundle",
                    transpose=True, bg=[0] if name == "breakfast" else [10],
                    avg_len=6.9 if name == "breakfast" else 32.9)
    if name == "ego":
        root = f"{base}data/egoprocel/"
        return dict(mapping=root + "mapping.txt", root=root, features=root + "features/",
                    train=root + "%s.train" % cfg.split, test=root + "%s.test" % cfg.split,
                    transpose=False, bg=[0], avg_len=21.5 if o2o else 7.4)
    if name == "epic":
        root = f"{base}data/epic-kitchens/processed/"
        return dict(mapping=root + "mapping.txt", root=root, features=root + "features",
                    train=root + "%s.train" % cfg.split, test=root + "%s.test" % cfg.split,
                    transpose=False, bg=[0], avg_len=165 if o2o else 52)
    if name.startswith("havid"):
        variant = name.replace("havid_", "")
        hb = f"{base}data/HAViD/ActionSegmentation/data"
        root = f"{hb}/{variant}/"
        avg = 8.0 if variant.endswith("_pt") else 15.0 if variant.endswith("_aa") else 10.0
        return dict(mapping=f"{root}mapping.txt", root=root, features=f"{hb}/features",
                    train=f"{root}splits/train.{cfg.split}.bundle", test=f"{root}splits/test.{cfg.split}.bundle",
                    transpose=True, bg=[0], avg_len=avg)
    raise ValueError(f"unknown dataset {name!r}")


def create_dataset(cfg, base=None):
    """dataset.py:169-351: (train dataset, test dataset) for ``cfg.dataset`` / ``cfg.split``;
    ``cfg.sr`` > 1 subsamples features and majority-pools training labels; holdout mode drops
    training videos that contain a holdout class and records seen / holdout class lists."""
    base = get_project_base() if base is None else base.rstrip("/") + "/"
    spec = _dataset_spec(cfg, base)
    gt_path = os.path.join(spec["root"], "groundTruth")
    print("Loading Feature from", spec["features"])
    print("Loading Label from", gt_path)
    label2index, index2label = load_action_mapping(spec["mapping"])
    nclasses = len(label2index)

    def load_video(vname):
        feature = load_feature(spec["features"], vname, spec["transpose"])
        with open(os.path.join(gt_path, vname + ".txt")) as f:
            gt_label = [label2index[line] for line in f.read().split("\n")[:-1]]
        n = min(feature.shape[0], len(gt_label))
        feature, gt_label = feature[:n], gt_label[:n]
        if cfg.sr > 1:
            return feature[::cfg.sr], shrink_frame_label(gt_label, cfg.sr), gt_label
        return feature, gt_label, gt_label

    strip = cfg.dataset in ("breakfast", "50salads", "gtea") or cfg.dataset.startswith("havid")
    txt_only = cfg.dataset.startswith("havid")
    test_list = _read_split(spec["test"], strip, txt_only)
    test_dataset = Dataset(test_list, nclasses, load_video, spec["bg"])

    if cfg.aux.debug:
        dataset = test_dataset
    else:
        video_list = _read_split(spec["train"], strip, txt_only)
        if cfg.holdout_mode and len(cfg.holdout_classes) > 0:
            holdout = list(cfg.holdout_classes)
            n0 = len(video_list)
            keep = [v for v in video_list if not video_contains_holdout_classes(v, gt_path, label2index, holdout)]
            print(f"HOLDOUT MODE: classes {holdout} "
                  f"({[index2label[c] for c in holdout if c in index2label]}); "
                  f"training videos {n0} -> {len(keep)}")
            video_list = keep
            if len(video_list) == 0:
                raise ValueError("No training videos remaining after holdout filtering!")
        dataset = Dataset(video_list, nclasses, load_video, spec["bg"])

    holdout_on = cfg.holdout_mode and len(cfg.holdout_classes) > 0
    holdout = list(cfg.holdout_classes) if holdout_on else []
    seen = [c for c in range(nclasses) if c not in holdout]
    for d in (dataset, test_dataset):
        d.average_transcript_len = spec["avg_len"]
        d.label2index = label2index
        d.index2label = index2label
        d.holdout_classes = list(holdout)
        d.seen_classes = list(seen)
    return dataset, test_dataset
