"""Drop-in for the reference's Python module ``protocols``
(simulator/gym/cpr_gym_engine.ml:165-304): constructors returning protocol specs that
``engine.create`` accepts. Nakamoto, Ethereum, B_k and Tailstorm run as lockstep lanes on the
device engine; the other constructors (SPar, STree, SDag, TailstormJune: outside the north
star) exist with the reference's signatures and raise.
"""

from . import _lib as L


class Protocol:
    """Stands in for the reference's "ocaml.protocol" capsule."""

    def __init__(self, key, description, attack_info, unit_observation,
                 protocol_id=L.PROTO_NAKAMOTO, **params):
        self.key = key
        self.protocol_id = protocol_id
        self.description = description
        self.attack_info = attack_info
        self.unit_observation = bool(unit_observation)
        self.params = params

    def __repr__(self):
        return f"<cpr_amd protocol {self.key} ({self.attack_info})>"


def nakamoto(unit_observation):
    # nakamoto.ml:3-4 (key, description), nakamoto_ssz.ml:15-21 (attack-space info)
    info = "SSZ'16 attack space with %s observations" % ("unit" if unit_observation else "raw")
    return Protocol("nakamoto", "Nakamoto consensus", info, unit_observation)


def _not_on_device(name):
    def ctor(*args, **kwargs):
        raise NotImplementedError(
            f"protocols.{name}: not implemented by the device engine (it covers Nakamoto, "
            "Ethereum, B_k and Tailstorm; DESIGN.md §8)"
        )

    ctor.__name__ = name
    return ctor


def _option(choice, value):
    # options.ml:56-77 of_string_exn: "'x' is not a valid parameter choice, try 'a' or 'b'"
    if value in choice:
        return value
    quoted = [f"'{c}'" for c in choice]
    alts = quoted[0] if len(quoted) == 1 else ", ".join(quoted[:-1]) + " or " + quoted[-1]
    raise ValueError(f"'{value}' is not a valid parameter choice, try {alts}")


def ethereum(reward, unit_observation):
    """ethereum_ssz attack space over Byzantium parameters with the chosen incentive scheme
    (cpr_gym_engine.ml:180-192, cpr_protocols.ml:39-49, ethereum.ml:19-55)."""
    reward = _option(["constant", "discount"], reward)  # ethereum.ml:3 incentive_schemes
    info = "SSZ'16-like attack space with %s observations" % ("unit" if unit_observation else "raw")
    # ethereum.ml:29-55: key / description over (preference, progress, max_uncles, scheme)
    return Protocol(f"eth-heaviest_chain-work-2-{reward}",
                    f"Ethereum with heaviest_chain-preference, work-progress, uncle cap 2, "
                    f"and {reward}-rewards", info, unit_observation,
                    protocol_id=L.PROTO_ETHEREUM, reward=reward,
                    reward_scheme=L.REWARD_DISCOUNT if reward == "discount" else L.REWARD_CONSTANT)


def bk(reward, k, unit_observation):
    """bk_ssz attack space over B_k (cpr_gym_engine.ml:193-206, cpr_protocols.ml:53-72)."""
    reward = _option(["block", "constant"], reward)  # bk.ml:3 incentive_schemes
    k = int(k)
    if k < 1:
        raise ValueError("k must be positive")
    info = "SSZ'16-like attack space with %s observations" % ("unit" if unit_observation else "raw")
    return Protocol(f"bk-{k}-{reward}", f"Bₖ with k={k} and {reward} rewards", info,
                    unit_observation, protocol_id=L.PROTO_BK, k=k, reward=reward,
                    reward_scheme=L.REWARD_BLOCK if reward == "block" else L.REWARD_CONSTANT)

spar = _not_on_device("spar")
stree = _not_on_device("stree")
sdag = _not_on_device("sdag")


def tailstorm(reward, k, subblock_selection, unit_observation):
    """tailstorm_ssz attack space (cpr_gym_engine.ml:245-265, cpr_protocols.ml:153-175)."""
    reward = _option(["constant", "discount", "punish", "hybrid"], reward)  # tailstorm.ml:3
    subblock_selection = _option(["altruistic", "heuristic", "optimal"], subblock_selection)
    k = int(k)
    if k < 1:
        raise ValueError("k must be positive")
    info = "SSZ'16-like attack space with %s observations" % ("unit" if unit_observation else "raw")
    desc = (f"Tailstorm with k={k}, {reward} rewards, and {subblock_selection} "
            "sub-block selection")  # tailstorm.ml:35-43
    scheme = {"constant": L.REWARD_CONSTANT, "discount": L.REWARD_DISCOUNT,
              "punish": L.REWARD_PUNISH, "hybrid": L.REWARD_HYBRID}[reward]
    sel = {"altruistic": L.SELECT_ALTRUISTIC, "heuristic": L.SELECT_HEURISTIC,
           "optimal": L.SELECT_OPTIMAL}[subblock_selection]
    return Protocol(f"tailstorm-{k}-{reward}-{subblock_selection}", desc, info, unit_observation,
                    protocol_id=L.PROTO_TAILSTORM, k=k, reward=reward, reward_scheme=scheme,
                    subblock_selection=subblock_selection, selection_id=sel)

tailstormjune = _not_on_device("tailstormjune")
