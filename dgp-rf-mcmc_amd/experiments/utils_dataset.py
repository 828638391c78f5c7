"""Data loading of the reference's experiments/utils_dataset.py + datasets.py, device-resident.

A `DeviceDataset` plays the role of the reference's `tf.data.Dataset` pipelines
(from_tensor_slices -> map -> shuffle -> batch(drop_remainder) [-> repeat]): the whole split lives
in HBM once, each pass draws a fresh permutation on the device and yields device views of the
minibatches.  The samplers in utils_training.py read `ds.X / ds.Y / ds.batch_size` to run whole
epochs as hipGraph replays with the minibatch permutation drawn inside the step kernels.

UCI data is read from `{data_dir}{name}.csv` (last column = y) exactly like the reference's
`Dataset.read_data`; there is no network here, so nothing is downloaded (`download_data` raises).
"""
import os

import numpy as np
import torch

from dgprf import engine as E


# ----------------------------------------------------------------------------- datasets.py
class Dataset(object):
    """experiments/datasets.py:31-87: CSV read, seeded 90/10 split, train-statistics
    normalisation of X (std + 1e-6) and of Y (mean only: the reference divides Y by 1)."""

    def __init__(self, name, N, D, type, data_path='/data/'):
        self.data_path = data_path
        self.name, self.N, self.D = name, N, D
        assert type in ['regression', 'classification', 'multiclass']
        self.type = type

    def csv_file_path(self, name):
        return '{}{}.csv'.format(self.data_path, name)

    def read_data(self):
        data = np.loadtxt(self.csv_file_path(self.name), delimiter=',', ndmin=2)
        return {'X': data[:, :-1], 'Y': data[:, -1, None]}

    def download_data(self):
        raise FileNotFoundError(
            f"{self.csv_file_path(self.name)} not found and there is no network to download "
            f"UCI '{self.name}' (experiments/datasets.py download_data); place the CSV there")

    def get_data(self, seed=0, split=0, prop=0.9):
        path = self.csv_file_path(self.name)
        if not os.path.isfile(path):
            self.download_data()
        full_data = self.read_data()
        split_data = self.split(full_data, seed, split, prop)
        split_data = self.normalize(split_data, 'X')
        if self.type == 'regression':
            split_data = self.normalize(split_data, 'Y')
        return split_data

    def split(self, full_data, seed, split, prop):
        """datasets.py:58-72 — the legacy global numpy RNG, so the index split is bit-exact."""
        ind = np.arange(self.N)
        np.random.seed(seed + split)
        np.random.shuffle(ind)
        n = int(self.N * prop)
        return {'X': full_data['X'][ind[:n], :], 'Xs': full_data['X'][ind[n:], :],
                'Y': full_data['Y'][ind[:n], :], 'Ys': full_data['Y'][ind[n:], :]}

    def normalize(self, split_data, X_or_Y):
        """datasets.py:74-87.  The reference never stores 'Y_std' (Y is divided by 1) while
        utils_dataset.py:20 reads it (a KeyError there); the divisor actually used, 1, is
        recorded as Y_std so the samplers' 'restore via Y_std' is the identity it implies."""
        m = np.average(split_data[X_or_Y], 0)[None, :]
        if X_or_Y == "X":
            s = np.std(split_data[X_or_Y], 0)[None, :] + 1e-6
        else:
            s = 1.
        split_data[X_or_Y] = (split_data[X_or_Y] - m) / s
        split_data[X_or_Y + 's'] = (split_data[X_or_Y + 's'] - m) / s
        split_data.update({X_or_Y + '_mean': m.flatten()})
        if X_or_Y == "X":
            split_data.update({X_or_Y + '_std': s.flatten()})
        else:
            split_data.update({'Y_std': np.ones(np.shape(m.flatten()))})
        return split_data


_UCI = [('boston', 506, 13), ('concrete', 1030, 8), ('energy', 768, 8), ('kin8nm', 8192, 8),
        ('naval', 11934, 12), ('power', 9568, 4), ('protein', 45730, 9), ('wine_red', 1599, 11),
        ('wine_white', 4898, 11)]  # datasets.py:94-234 (name, N, D)


class Datasets(object):
    """datasets.py:237-257: every UCI regression set by name."""

    def __init__(self, data_path='/data/'):
        self.all_datasets = {}
        for name, N, D in _UCI:
            self.all_datasets[name] = Dataset(name, N, D, 'regression', data_path=data_path)


# ----------------------------------------------------------------------------- tf.data stand-in
class DeviceDataset:
    """The reference's tf.data pipeline over (X, Y) held in HBM.

    from_tensor_slices + map + shuffle(full buffer) + batch(B, drop_remainder) [+ repeat]; every
    iteration of a shuffled dataset draws a new permutation (tf's reshuffle_each_iteration)."""

    def __init__(self, X, Y, batch_size=None, drop_remainder=False, shuffle=False,
                 repeat=False, seed=None, dev=None):
        dev = dev or E.device()
        self.X = E.as_device(X, dev)
        Y = E.as_device(Y, dev)
        self.Y = Y[:, None] if Y.dim() == 1 else Y
        if self.X.shape[0] != self.Y.shape[0]:
            raise ValueError("X and Y must have the same number of rows")
        self.batch_size = batch_size
        self.drop_remainder = bool(drop_remainder)
        self.shuffled = bool(shuffle)
        self.repeated = bool(repeat)
        self.seed = int(np.random.randint(2**31 - 1)) if seed is None else int(seed)
        self._pass = 0

    @classmethod
    def from_tensor_slices(cls, XY, dev=None):
        X, Y = XY
        return cls(X, Y, dev=dev)

    def _copy(self, **kw):
        d = DeviceDataset.__new__(DeviceDataset)
        d.__dict__.update(self.__dict__)
        d.__dict__.update(kw)
        d._pass = 0
        return d

    def map(self, fn):
        """Element-wise transform applied once to the resident arrays (fn must accept a batch)."""
        X, Y = fn(self.X, self.Y)
        return self._copy(X=X, Y=Y if Y.dim() == 2 else Y[:, None])

    def shuffle(self, buffer_size=None, seed=None):
        return self._copy(shuffled=True, seed=self.seed if seed is None else int(seed))

    def batch(self, batch_size, drop_remainder=False):
        return self._copy(batch_size=int(batch_size), drop_remainder=bool(drop_remainder))

    def repeat(self):
        return self._copy(repeated=True)

    @property
    def n(self):
        return int(self.X.shape[0])

    def num_batches(self):
        B = self.batch_size or self.n
        return self.n // B if self.drop_remainder else -(-self.n // B)

    def __len__(self):
        return self.num_batches()

    def _one_pass(self):
        B = self.batch_size or self.n
        nb = self.num_batches()
        if self.shuffled:
            g = torch.Generator(device=self.X.device)
            g.manual_seed(self.seed * 1000003 + self._pass)
            perm = torch.randperm(self.n, generator=g, device=self.X.device)
        self._pass += 1
        for i in range(nb):
            lo, hi = i * B, min((i + 1) * B, self.n)
            if self.shuffled:
                idx = perm[lo:hi]
                yield self.X.index_select(0, idx), self.Y.index_select(0, idx)
            else:
                yield self.X[lo:hi], self.Y[lo:hi]

    def __iter__(self):
        if not self.repeated:
            yield from self._one_pass()
            return
        while True:
            yield from self._one_pass()


# ----------------------------------------------------------------------------- utils_dataset.py
def transform_UCI_tfds(X_train, Y_train, X_test, Y_test):
    """utils_dataset.py:7-14."""
    return (DeviceDataset.from_tensor_slices((X_train, Y_train)),
            DeviceDataset.from_tensor_slices((X_test, Y_test)))


def download_UCI_data_info(name, data_path='./data/'):
    """utils_dataset.py:16-24: (X, Y, Xs, Ys, X_mean, Y_mean, Y_std) as float32."""
    datasets = Datasets(data_path=data_path)
    dataset = datasets.all_datasets[name]
    data = dataset.get_data()
    X, Y, Xs, Ys, X_mean, Y_mean, Y_std = [np.float32(data[_]) for _ in
                                           ['X', 'Y', 'Xs', 'Ys', 'X_mean', 'Y_mean', 'Y_std']]
    assert dataset.N == X.shape[0] + Xs.shape[0], \
        f"N + Ns does not match dataset.N (should be {X.shape[0] + Xs.shape[0]})! "
    assert dataset.D == X.shape[1], f"D does not match dataset.D(should be {X.shape[1]})!"
    return X, Y, Xs, Ys, X_mean, Y_mean, Y_std


def load_arrays(X, Y, Xs, Ys, batch_size=128, transform_fn=None, drop_train_remainder=True):
    """The pipeline of load_UCI_dataset over arrays already in memory: shuffled train batches
    (drop_remainder), test batches in a FIXED order.  (The reference also shuffles the test set on
    every pass, utils_dataset.py:36, which misaligns the test points of the [S, N] log-likelihood
    matrix between samples before its logsumexp over S; keeping the order fixed is the intended
    computation.)"""
    ds_train, ds_test = transform_UCI_tfds(X, Y, Xs, Ys)
    if transform_fn is not None:
        ds_train = ds_train.map(transform_fn)
        ds_test = ds_test.map(transform_fn)
    ds_train = ds_train.shuffle(ds_train.n)
    ds_train = ds_train.batch(batch_size, drop_remainder=drop_train_remainder)
    ds_test = ds_test.batch(batch_size, drop_remainder=False)
    return ds_train, ds_test, tuple(np.shape(X)), tuple(np.shape(Xs))


def load_UCI_dataset(dataset_name, batch_size=128, transform_fn=None, data_dir='./data/',
                     drop_train_remainder=True):
    """utils_dataset.py:26-44 -> (ds_train, ds_test, train_shape, test_shape)."""
    print('#' * 30 + f" Getting data info:dataset name: {dataset_name} " + '#' * 30)
    X, Y, Xs, Ys, X_mean, Y_mean, Y_std = download_UCI_data_info(dataset_name, data_path=data_dir)
    print(f"D: {X.shape[1]}, N: {X.shape[0]}, Ns: {Xs.shape[0]}")
    print(f"X_mean: {X_mean}, Y_mean: {Y_mean}, Y_std: {Y_std}")
    print('#' * 70)
    return load_arrays(X, Y, Xs, Ys, batch_size, transform_fn, drop_train_remainder)


def load_tf_dataset(dataset_name, batch_size=128, transform_fn=None,
                    data_dir='./tensorflow_datasets/'):
    """utils_dataset.py:46-60.  tensorflow_datasets is not available; a local
    `{data_dir}{dataset_name}.npz` with arrays x_train, y_train, x_test, y_test (loaded with
    allow_pickle=False) stands in for tfds.load(...)."""
    path = os.path.join(data_dir, f"{dataset_name}.npz")
    if not os.path.isfile(path):
        raise FileNotFoundError(f"{path} not found (tensorflow_datasets is not available here)")
    with np.load(path, allow_pickle=False) as f:
        X, Y, Xs, Ys = f["x_train"], f["y_train"], f["x_test"], f["y_test"]
    ds_train, ds_test, tr_shape, te_shape = load_arrays(X, Y, Xs, Ys, batch_size, transform_fn,
                                                        drop_train_remainder=True)
    return ds_train, ds_test, tr_shape[0], te_shape[0]


def normalize_MNIST(img, label):
    """utils_dataset.py:62-65, on a batch: [n, 28, 28] uint8 -> [n, 784] / 255 - 0.5; label [n, 1]."""
    img = torch.as_tensor(img)
    n = img.shape[0]
    img = img.reshape(n, 28 * 28).to(torch.float32) / 255. - 0.5
    label = torch.as_tensor(label).reshape(n, 1).to(torch.float32)
    return img, label
