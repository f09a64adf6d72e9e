"""Drop-in for the reference's Python module ``protocols``
(simulator/gym/cpr_gym_engine.ml:438-577): constructors returning protocol specs that
``engine.create`` accepts. Only Nakamoto + SSZ'16 attack space runs on the device engine
in this build; the other constructors exist with the reference's signatures and raise.
"""


class Protocol:
    """Stands in for the reference's "ocaml.protocol" capsule."""

    def __init__(self, key, description, attack_info, unit_observation, **params):
        self.key = key
        self.description = description
        self.attack_info = attack_info
        self.unit_observation = bool(unit_observation)
        self.params = params

    def __repr__(self):
        return f"<cpr_amd protocol {self.key} ({self.attack_info})>"


def nakamoto(unit_observation):
    # nakamoto.ml:3-4 (key, description), nakamoto_ssz.ml:115-121 (attack-space info)
    info = "SSZ'16 attack space with %s observations" % ("unit" if unit_observation else "raw")
    return Protocol("nakamoto", "Nakamoto consensus", info, unit_observation)


def _not_on_device(name):
    def ctor(*args, **kwargs):
        raise NotImplementedError(
            f"protocols.{name}: the device engine implements Nakamoto only in this build "
            "(see DESIGN.md §8, next rows: Ethereum, B_k, Tailstorm)"
        )

    ctor.__name__ = name
    return ctor


ethereum = _not_on_device("ethereum")  # (reward, unit_observation)
bk = _not_on_device("bk")  # (reward, k, unit_observation)
spar = _not_on_device("spar")
stree = _not_on_device("stree")
sdag = _not_on_device("sdag")
tailstorm = _not_on_device("tailstorm")  # (reward, k, subblock_selection, unit_observation)
tailstormjune = _not_on_device("tailstormjune")
