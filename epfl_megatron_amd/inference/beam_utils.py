"""n-best list for beam search (reference ``megatron/text_generation/beam_utils.py``)."""
import heapq


class BeamHypotheses:
    """Keeps the ``num_beams`` best finished hypotheses by length-normalised
    log-probability ``sum_logprobs / length ** length_penalty``."""

    def __init__(self, num_beams, length_penalty=1.0, early_stopping=False):
        self.num_beams = num_beams
        self.length_penalty = length_penalty
        self.early_stopping = early_stopping
        self._heap = []  # (score, counter, hyp) min-heap
        self._n = 0

    @property
    def beams(self):
        return [(s, h) for s, _, h in self._heap]

    @property
    def worst_score(self):
        return self._heap[0][0] if len(self._heap) >= self.num_beams else 1e9

    def __len__(self):
        return len(self._heap)

    def add(self, hyp, sum_logprobs, length):
        score = float(sum_logprobs) / (length ** self.length_penalty)
        self._n += 1
        if len(self._heap) < self.num_beams:
            heapq.heappush(self._heap, (score, self._n, hyp))
        elif score > self._heap[0][0]:
            heapq.heapreplace(self._heap, (score, self._n, hyp))

    def is_done(self, best_sum_logprobs, cur_len):
        if len(self) < self.num_beams:
            return False
        if self.early_stopping:
            return True
        return self._heap[0][0] >= best_sum_logprobs / cur_len ** self.length_penalty
