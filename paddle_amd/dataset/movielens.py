"""MovieLens 1M (reference python/paddle/dataset/movielens.py).  Reads
``DATA_HOME/movielens/ml-1m.zip`` (``movies.dat`` / ``users.dat`` / ``ratings.dat``,
``::``-separated, latin-1).  Sample: [user id, gender (0 M / 1 F), age bucket, job,
movie id, [category ids], [title word ids], [rating * 2 - 5]]; ratings are split
train / test by a seeded uniform draw (test_ratio 0.1).  Category and title-word
ids are assigned in sorted order (deterministic).  Without the archive: synthetic
samples of the same layout."""
from __future__ import annotations

import functools
import re
import zipfile

import numpy as np

from . import common

URL = "http://files.grouplens.org/datasets/movielens/ml-1m.zip"
MD5 = "c4d9eecfca2ab87c1945afe126590906"
age_table = [1, 18, 25, 35, 45, 50, 56]
_META = {}


class MovieInfo:
    def __init__(self, index, categories, title):
        self.index, self.categories, self.title = int(index), categories, title

    def value(self):
        return [self.index, [_META["cat"][c] for c in self.categories],
                [_META["title"][w.lower()] for w in self.title.split()]]


class UserInfo:
    def __init__(self, index, gender, age, job_id):
        self.index, self.is_male = int(index), gender == "M"
        self.age, self.job_id = age_table.index(int(age)), int(job_id)

    def value(self):
        return [self.index, 0 if self.is_male else 1, self.age, self.job_id]


def _read(pkg, name):
    with pkg.open(name) as f:
        for ln in f:
            yield ln.decode("latin-1").strip()


def _meta(path):
    if _META.get("path") == path:
        return
    title_re = re.compile(r"^(.*)\((\d+)\)$")
    movies, cats, words = {}, set(), set()
    with zipfile.ZipFile(path) as pkg:
        for ln in _read(pkg, "ml-1m/movies.dat"):
            mid, title, cat = ln.split("::")
            m = title_re.match(title)
            title = m.group(1) if m else title
            c = cat.split("|")
            movies[int(mid)] = MovieInfo(mid, c, title)
            cats.update(c)
            words.update(w.lower() for w in title.split())
        users = {}
        for ln in _read(pkg, "ml-1m/users.dat"):
            uid, g, age, job, _ = ln.split("::")
            users[int(uid)] = UserInfo(uid, g, age, job)
    _META.update(path=path, movies=movies, users=users, cat={c: i for i, c in enumerate(sorted(cats))},
                 title={w: i for i, w in enumerate(sorted(words))})


def _reader(rand_seed=0, test_ratio=0.1, is_test=False):
    path = common.download(URL, "movielens", MD5)
    if path is None:
        common.synthetic_notice("movielens", "ml-1m.zip")
        rng = np.random.RandomState(2 if is_test else 1)
        for _ in range(1000 if is_test else 9000):
            yield [int(rng.randint(1, 6041)), int(rng.randint(0, 2)), int(rng.randint(0, 7)), int(rng.randint(0, 21)),
                   int(rng.randint(1, 3953)), [int(rng.randint(0, 18))], [int(x) for x in rng.randint(0, 5175, 4)],
                   [float(rng.randint(1, 6)) * 2 - 5.0]]
        return
    _meta(path)
    rng = np.random.RandomState(rand_seed)
    with zipfile.ZipFile(path) as pkg:
        for ln in _read(pkg, "ml-1m/ratings.dat"):
            if (rng.random_sample() < test_ratio) != is_test:
                continue
            uid, mid, rating, _ = ln.split("::")
            yield (_META["users"][int(uid)].value() + _META["movies"][int(mid)].value()
                   + [[float(rating) * 2 - 5.0]])


def _creator(**kw):
    return lambda: _reader(**kw)


train = functools.partial(_creator, is_test=False)
test = functools.partial(_creator, is_test=True)


def _need_meta():
    path = common.download(URL, "movielens", MD5)
    if path is None:
        raise RuntimeError(f"movielens metadata needs {common.DATA_HOME}/movielens/ml-1m.zip")
    _meta(path)


def get_movie_title_dict():
    _need_meta()
    return _META["title"]


def movie_categories():
    _need_meta()
    return _META["cat"]


def max_movie_id():
    _need_meta()
    return max(_META["movies"])


def max_user_id():
    _need_meta()
    return max(_META["users"])


def max_job_id():
    _need_meta()
    return max(u.job_id for u in _META["users"].values())


def user_info():
    _need_meta()
    return _META["users"]


def movie_info():
    _need_meta()
    return _META["movies"]


def fetch():
    return common.download(URL, "movielens", MD5)
