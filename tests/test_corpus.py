"""CPU: synthetic corpus generator against the survey's SHA-256 values."""
import hashlib

import pytest

import dmx

SHA_1MIB = {
    "zeros": "30e14955ebf1352266dc2ff8067e68104607e750abb9d3b36582b8af909fcb58",
    "repeat": "b7caea828d5414a3ea9d55cc9dfd9ac14000778c48ee07b53344d6127d618c2b",
    "random": "ebf19c93a5201f443514faf086179df750164be00157084581113fd5dc2063e5",
    "text": "afd7235285ec5ed8cfe57317b5cabbe24c74bbb74117e3c74b97930d18d052cf",
    "mixed": "9c57f3001acd34409473b59656501d667cae6fb143faccf8a9616e8f2c69ccec",
}


@pytest.mark.parametrize("kind", sorted(SHA_1MIB))
def test_corpus_sha256(kind):
    assert hashlib.sha256(dmx.corpus(kind, 1 << 20)).hexdigest() == SHA_1MIB[kind]


def test_bmp_full_file_sha256():
    d = dmx.corpus("bmp", 25165962)
    assert hashlib.sha256(d).hexdigest() == "67eefcfa5d39b09aadafefe3e690f5e43bfc0382888671fa55a3ec9f4c1d7f5a"


@pytest.mark.parametrize("kind", ["repeat", "random", "text", "mixed", "bmp"])
def test_corpus_windows_are_prefix_stable(kind):
    full = dmx.corpus(kind, 300000)
    assert dmx.corpus(kind, 70001, offset=123457) == full[123457:123457 + 70001]
