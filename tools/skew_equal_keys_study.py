"""Study (not product code): the pop order of equal-time events in orderedQueue.ml's skew
heap (insertion: a new element that is not smaller swaps the node's children and goes down
the new left side; deletion: the root's children merged, ties taken from the left), the
structure every event engine here replays exactly. Starting from a heap that holds a later
element (the next clock), random interleavings of pushes and pops of equal-time events are
compared with FIFO and LIFO order. They match neither: the order depends on the heap's
shape, so a window whose events share an instant (every window of the two-agents network,
the activation instant of every B_k window) cannot drop the heap.

usage: python tools/skew_equal_keys_study.py [trials]
"""
import random
import sys


class Node:
    __slots__ = ("t", "v", "l", "r")

    def __init__(self, t, v):
        self.t, self.v, self.l, self.r = t, v, None, None


def push(h, t, v):
    if h is None:
        return Node(t, v)
    root, node, parent = h, h, None
    while True:
        if node is None:
            parent.l = Node(t, v)
            return root
        if t < node.t:  # the new element takes the node, the old one moves down
            node.t, t = t, node.t
            node.v, v = v, node.v
        else:
            node.l, node.r = node.r, node.l
        parent, node = node, node.l


def pop(h):
    v = h.v
    node, parent, side, root = h, None, 0, h
    while True:
        l, r = node.l, node.r
        if r is None or l is None:
            repl = l if r is None else r
            if parent is None:
                root = repl
            elif side == 0:
                parent.l = repl
            else:
                parent.r = repl
            return v, root
        if l.t <= r.t:
            node.t, node.v = l.t, l.v
            parent, side, node = node, 0, l
        else:
            node.t, node.v = r.t, r.v
            parent, side, node = node, 1, r


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    rnd = random.Random(1)
    kinds = {"fifo": 0, "lifo": 0, "other": 0}
    for _ in range(trials):
        h = push(None, 1.0, "clock")
        pushed, out, c = [], [], 0
        for _ in range(rnd.randrange(3, 40)):
            if rnd.random() < 0.6 or h.t > 0:
                h = push(h, 0.0, c)
                pushed.append(c)
                c += 1
            else:
                v, h = pop(h)
                out.append(v)
        while h is not None and h.t == 0:
            v, h = pop(h)
            out.append(v)
        kinds["fifo" if out == pushed else "lifo" if out == pushed[::-1] else "other"] += 1
    print(kinds)


if __name__ == "__main__":
    main()
