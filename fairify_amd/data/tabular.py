"""Tabular dataset loaders reproducing the reference encodings (C04) + synthetic data.

Reference loaders: ``load_adult_ac1`` (utils/verif_utils.py:119-190), ``load_german``
(:193-241, with ``german_custom_preprocessing`` utils/standard_data.py:4-65),
``load_compass`` (:243-265), ``load_default`` (:267-307), ``load_bank`` (:309-366).
Semantics kept: LabelEncoder codes (sorted unique values), KBins(20, uniform) for Adult
capital-gain/loss, binarised German age (>= 26) and Bank age (>= 25), German code grouping
and ``sex`` derived from ``personal_status``, one-hot(drop first)+MinMax for Default,
85/15 split with seed 42.  Fixed: the removed ``np.float`` alias
(utils/verif_utils.py:204,325); Bank falls back to ``bank-additional.csv`` because the
``-full`` file is not shipped (.MISSING_LARGE_BLOBS:1).

The data root is ``$FAIRIFY_DATA`` or ``/root/reference/data``; when absent (e.g. on a
benchmark box) :func:`synthetic` generates labelled rows of the same integer domain.
"""
from __future__ import annotations

import os
import warnings
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np
import pandas as pd

from ..spec import DOMAINS, Domain


def data_root() -> str:
    return os.environ.get("FAIRIFY_DATA", "/root/reference/data")


@dataclass
class Dataset:
    name: str
    df: pd.DataFrame
    X_train: np.ndarray
    y_train: np.ndarray
    X_test: np.ndarray
    y_test: np.ndarray
    columns: list
    label: str
    encoders: Dict = field(default_factory=dict)
    synthetic: bool = False


def _split(df: pd.DataFrame, label: str, name: str, encoders=None) -> Dataset:
    from sklearn.model_selection import train_test_split

    X = df.drop(columns=[label])
    y = df[label]
    Xtr, Xte, ytr, yte = train_test_split(X, y, test_size=0.15, random_state=42)
    return Dataset(name, df, Xtr.to_numpy(dtype=np.float64), ytr.to_numpy().astype(int), Xte.to_numpy(dtype=np.float64),
                   yte.to_numpy().astype(int), list(X.columns), label, encoders or {})


def _label_encode(df: pd.DataFrame, cols, encoders):
    from sklearn.preprocessing import LabelEncoder

    for c in cols:
        le = LabelEncoder()
        df[c] = le.fit_transform(df[c])
        encoders[c] = le


def load_adult(root: Optional[str] = None) -> Dataset:
    from sklearn.preprocessing import KBinsDiscretizer

    root = root or data_root()
    cols = ['age', 'workclass', 'fnlwgt', 'education', 'education-num', 'marital-status', 'occupation',
            'relationship', 'race', 'sex', 'capital-gain', 'capital-loss', 'hours-per-week', 'native-country',
            'income-per-year']
    train = pd.read_csv(os.path.join(root, "adult", "adult.data"), header=None, names=cols, skipinitialspace=True,
                        na_values=['?'])
    test = pd.read_csv(os.path.join(root, "adult", "adult.test"), header=0, names=cols, skipinitialspace=True,
                       na_values=['?'])
    df = pd.concat([test, train], ignore_index=True).drop(columns=['fnlwgt']).dropna()
    enc: Dict = {}
    _label_encode(df, ['sex', 'workclass', 'education', 'marital-status', 'occupation', 'relationship',
                       'native-country', 'race'], enc)
    for c in ['capital-gain', 'capital-loss']:
        kb = KBinsDiscretizer(n_bins=20, encode='ordinal', strategy='uniform')
        df[c] = kb.fit_transform(df[[c]])
        enc[c] = kb
    lab = 'income-per-year'
    df[lab] = df[lab].isin(['>50K', '>50K.']).astype(int)
    return _split(df, lab, "adult", enc)


_GERMAN_COLS = ['status', 'month', 'credit_history', 'purpose', 'credit_amount', 'savings', 'employment',
                'investment_as_income_percentage', 'personal_status', 'other_debtors', 'residence_since',
                'property', 'age', 'installment_plans', 'housing', 'number_of_credits', 'skill_level',
                'people_liable_for', 'telephone', 'foreign_worker', 'credit']


def german_preprocess(df: pd.DataFrame) -> pd.DataFrame:
    """Code grouping + ``sex`` from ``personal_status`` (utils/standard_data.py:4-65)."""
    hist = {'A30': 'None/Paid', 'A31': 'None/Paid', 'A32': 'None/Paid', 'A33': 'Delay', 'A34': 'Other'}
    emp = {'A71': 'Unemployed', 'A72': '1-4 years', 'A73': '1-4 years', 'A74': '4+ years', 'A75': '4+ years'}
    sav = {'A61': '<500', 'A62': '<500', 'A63': '500+', 'A64': '500+', 'A65': 'Unknown/None'}
    sta = {'A11': '<200', 'A12': '<200', 'A13': '200+', 'A14': 'None'}
    sex = {'A91': 1, 'A93': 1, 'A94': 1, 'A92': 0, 'A95': 0}
    src = 'personal_status' if 'personal_status' in df.columns else 'sex'
    df['sex'] = df[src].map(lambda v: sex.get(v, v))
    df['credit_history'] = df['credit_history'].map(lambda v: hist.get(v, 'NA'))
    df['savings'] = df['savings'].map(lambda v: sav.get(v, 'NA'))
    df['employment'] = df['employment'].map(lambda v: emp.get(v, 'NA'))
    df['status'] = df['status'].map(lambda v: sta.get(v, 'NA'))
    if 'credit' in df.columns:
        df['credit'] = df['credit'].replace({1: 1, 2: 0})
    return df


def load_german(root: Optional[str] = None) -> Dataset:
    root = root or data_root()
    df = pd.read_csv(os.path.join(root, "german", "german.data"), sep=' ', header=None, names=_GERMAN_COLS)
    df['age'] = (df['age'] >= 26).astype(float)
    df = german_preprocess(df).drop(columns=['personal_status'])
    enc: Dict = {}
    _label_encode(df, ['status', 'credit_history', 'purpose', 'savings', 'employment', 'other_debtors', 'property',
                       'installment_plans', 'housing', 'skill_level', 'telephone', 'foreign_worker'], enc)
    return _split(df, 'credit', "german", enc)


def load_bank(root: Optional[str] = None) -> Dataset:
    root = root or data_root()
    path = os.path.join(root, "bank", "bank-additional-full.csv")
    if not os.path.exists(path):
        alt = os.path.join(root, "bank", "bank-additional.csv")
        warnings.warn("bank-additional-full.csv not shipped with the reference; using bank-additional.csv")
        path = alt
    cols = ['age', 'job', 'marital', 'education', 'default', 'housing', 'loan', 'contact', 'month', 'day_of_week',
            'duration', 'emp.var.rate', 'campaign', 'pdays', 'previous', 'poutcome', 'y']
    df = pd.read_csv(path, sep=';', na_values=['unknown']).dropna()
    df['age'] = (df['age'] >= 25).astype(float)
    enc: Dict = {}
    _label_encode(df, ['job', 'marital', 'education', 'default', 'housing', 'loan', 'contact', 'month',
                       'day_of_week', 'poutcome'], enc)
    df = df[cols].copy()
    df['y'] = (df['y'] == 'yes').astype(int)
    return _split(df, 'y', "bank", enc)


def load_compas(root: Optional[str] = None) -> Dataset:
    root = root or data_root()
    df = pd.read_csv(os.path.join(root, "compass", "compas_preprocessed_full.csv"))
    enc: Dict = {}
    _label_encode(df, ['Two_yr_Recidivism', 'Number_of_Priors', 'Age', 'Race', 'Female', 'Misdemeanor'], enc)
    return _split(df, 'score_factor', "compas", enc)


def load_default(root: Optional[str] = None) -> Dataset:
    from sklearn.preprocessing import MinMaxScaler, OneHotEncoder

    root = root or data_root()
    df = pd.read_csv(os.path.join(root, "default", "default.csv")).rename(columns={"PAY_0": "PAY_1"})
    df = df.drop(columns=["ID"])
    oh_cols = ["SEX", "EDUCATION", "MARRIAGE"]
    oh = OneHotEncoder(drop='first', sparse_output=False)
    enc_df = pd.DataFrame(oh.fit_transform(df[oh_cols]), columns=oh.get_feature_names_out(oh_cols))
    df = df.drop(columns=oh_cols).reset_index(drop=True).join(enc_df)
    pay = ["PAY_1", "PAY_2", "PAY_3", "PAY_4", "PAY_5", "PAY_6"]
    mm = MinMaxScaler()
    df[pay] = mm.fit_transform(df[pay])
    return _split(df, "default.payment.next.month", "default", {"onehot": oh, "minmax": mm})


LOADERS = {"adult": load_adult, "german": load_german, "bank": load_bank, "compas": load_compas,
           "default": load_default}


def synthetic(domain: Domain, n: int = 2000, seed: int = 0, mlp=None, label_noise: float = 0.0) -> Dataset:
    """Uniform integer rows of the domain; labels from ``mlp`` (if given) or a random linear rule."""
    rng = np.random.default_rng(seed)
    lo, hi = domain.lo(), domain.hi()
    X = rng.integers(lo, hi + 1, size=(n, domain.n)).astype(np.float64)
    if mlp is not None:
        y = mlp.predict(X)
    else:
        w = rng.normal(size=domain.n) / np.maximum(1, hi - lo)
        y = ((X - lo) @ w > np.median((X - lo) @ w)).astype(int)
    if label_noise:
        flip = rng.random(n) < label_noise
        y = np.where(flip, 1 - y, y)
    df = pd.DataFrame(X, columns=domain.names)
    df[domain.label] = y
    k = int(n * 0.85)
    return Dataset(f"synthetic-{domain.suite}", df, X[:k], y[:k], X[k:], y[k:], domain.names, domain.label,
                   synthetic=True)


def load(suite: str, root: Optional[str] = None, allow_synthetic: bool = True, seed: int = 0, mlp=None) -> Dataset:
    """Real dataset of a suite if present, otherwise synthetic rows of its domain."""
    key = "compas" if suite.startswith("compas") else suite
    try:
        if suite == "compas12":
            raise FileNotFoundError("no loader for the 12-feature COMPAS variant")
        return LOADERS[key](root)
    except (FileNotFoundError, KeyError, OSError):
        if not allow_synthetic:
            raise
        return synthetic(DOMAINS[suite], seed=seed, mlp=mlp)
