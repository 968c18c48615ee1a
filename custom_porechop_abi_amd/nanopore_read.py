"""Per-read adapter logic (mirror of porechop_abi/nanopore_read.py for the hot path).

Same class name, attribute names and method signatures as the reference, so the phase drivers
and the reference's own per-read call pattern work unchanged:
  * NanoporeRead.align_adapter_set   -- porechop_abi/nanopore_read.py:158-173
  * NanoporeRead.find_start_trim     -- :175-195
  * NanoporeRead.find_end_trim       -- :197-217
  * NanoporeRead.find_middle_adapters-- :219-252
  * NanoporeRead.determine_barcode   -- :408-482
  * align_adapter()                  -- :485-500
Every alignment runs on the GPU through cpp_function_wrappers.adapter_alignment (one pair per
call). The batched drivers in porechop_abi.py do the same work in bulk and then apply the SAME
decision rules through the _apply_* helpers below, so both paths share one implementation of
the trimming logic.

Trimmed output (get_fasta / get_fastq / get_split_read_parts, :66-156) is mirrored for the
per-read interface; the batched path writes through the native writer (misc.write_reads,
pcabi_reads_write). The verbose views the drivers print at verbosity 2 and 3
(formatted_start_seq ... middle_adapter_results, :254-406) give the reference's text, colour codes
included (tests/golden/g6_verbose.json.gz).
"""
from .cpp_function_wrappers import adapter_alignment
from .misc import END_FORMATTING, RED, YELLOW, red, yellow


_LOWER = 'abcdefghijklmnopqrstuvwxyz'   # what str.upper changes in an ASCII str


class NanoporeRead(object):

    def __init__(self, name, seq, quals):
        self.name = name
        # seq.upper(), and the RNA test count('U') > count('T') (nanopore_read.py:35-40): the same
        # values with memchr-speed membership scans where they decide it -- an ASCII read with no
        # lower-case letter is its own upper case, and a read without a U is not RNA (an 8 kb read:
        # ~35 -> ~5 us, most of building a batch of reads)
        seq_u = seq if seq.isascii() and not any(c in seq for c in _LOWER) else seq.upper()
        self.rna = 'U' in seq_u and seq_u.count('U') > seq_u.count('T')
        self.seq = seq_u.replace('U', 'T') if self.rna else seq_u
        self.quals = quals if len(quals) >= len(seq) else quals + '+' * (len(seq) - len(quals))

        self.start_trim_amount = 0
        self.end_trim_amount = 0
        self.start_adapter_alignments = []
        self.end_adapter_alignments = []

        self.middle_adapter_positions = set()
        self.middle_trim_positions = set()
        self.middle_hit_str = ''

        self.start_barcode_scores = {}
        self.end_barcode_scores = {}
        self.best_start_barcode = ('none', 0.0)
        self.best_end_barcode = ('none', 0.0)
        self.second_best_start_barcode = ('none', 0.0)
        self.second_best_end_barcode = ('none', 0.0)
        self.barcode_call = 'none'
        self.albacore_barcode_call = None

    # --- sequence views -------------------------------------------------------------------
    def adapters_found(self):
        """Fork filter (porechop_abi/nanopore_read.py:22-30): start AND end alignments found."""
        return bool(self.start_adapter_alignments) and bool(self.end_adapter_alignments)

    def get_seq_with_start_end_adapters_trimmed(self):
        if not self.start_trim_amount and not self.end_trim_amount:
            return self.seq
        return self.seq[self.start_trim_amount:len(self.seq) - self.end_trim_amount]

    def seq_length_with_start_end_adapters_trimmed(self):
        return len(self.get_seq_with_start_end_adapters_trimmed())

    def get_quals_with_start_end_adapters_trimmed(self):
        if not self.start_trim_amount and not self.end_trim_amount:
            return self.quals
        return self.quals[self.start_trim_amount:len(self.quals) - self.end_trim_amount]

    # --- trimmed output (porechop_abi/nanopore_read.py:84-156) ------------------------------
    def get_split_read_parts(self, min_split_read_size):
        """Maximal runs of the trimmed read outside middle_trim_positions, at least
        min_split_read_size long, as (seq, quals)."""
        seq = self.get_seq_with_start_end_adapters_trimmed()
        quals = self.get_quals_with_start_end_adapters_trimmed()
        parts, a = [], 0
        cut = self.middle_trim_positions
        for i in range(len(seq) + 1):
            if i == len(seq) or i in cut:
                if i > a:
                    parts.append((seq[a:i], quals[a:i]))
                a = i + 1
        return [x for x in parts if len(x[0]) >= min_split_read_size]

    def _output_parts(self, min_split_read_size, discard_middle, untrimmed):
        """(name, seq, quals) records get_fasta / get_fastq write, or None for ''."""
        if not self.middle_trim_positions:
            if untrimmed:
                seq, quals = self.seq, self.quals
            else:
                seq = self.get_seq_with_start_end_adapters_trimmed()
                quals = self.get_quals_with_start_end_adapters_trimmed()
            return [(self.name, seq, quals)] if seq else []
        if discard_middle:
            return []
        return [(add_number_to_read_name(self.name, i + 1), s, q)
                for i, (s, q) in enumerate(self.get_split_read_parts(min_split_read_size))]

    def get_fasta(self, min_split_read_size, discard_middle, untrimmed=False):
        out = []
        for name, seq, _ in self._output_parts(min_split_read_size, discard_middle, untrimmed):
            if self.rna:
                seq = seq.replace('T', 'U')
            out.append('>' + name + '\n' + ''.join(seq[p:p + 70] + '\n' for p in range(0, len(seq), 70)))
        return ''.join(out)

    def get_fastq(self, min_split_read_size, discard_middle, untrimmed=False):
        out = []
        for name, seq, quals in self._output_parts(min_split_read_size, discard_middle, untrimmed):
            if self.rna:
                seq = seq.replace('T', 'U')
            out.append('@' + name + '\n' + seq + '\n+\n' + quals + '\n')
        return ''.join(out)

    # --- hot path, one alignment per call --------------------------------------------------
    def align_adapter_set(self, adapter_set, end_size, scoring_scheme_vals):
        """Adapter-set discovery: raise the set's best start/end full-adapter identity."""
        if adapter_set.start_sequence:
            full = align_adapter(self.seq[:end_size], adapter_set.start_sequence[1], scoring_scheme_vals)[0]
            adapter_set.best_start_score = max(adapter_set.best_start_score, full)
        if adapter_set.end_sequence:
            full = align_adapter(self.seq[-end_size:], adapter_set.end_sequence[1], scoring_scheme_vals)[0]
            adapter_set.best_end_score = max(adapter_set.best_end_score, full)

    def find_start_trim(self, adapters, end_size, extra_trim_size, end_threshold,
                        scoring_scheme_vals, min_trim_size, check_barcodes, forward_or_reverse):
        window = self.seq[:end_size]
        for adapter in adapters:
            if not adapter.start_sequence:
                continue
            hit = align_adapter(window, adapter.start_sequence[1], scoring_scheme_vals)
            self._apply_start_hit(adapter, hit, end_size, extra_trim_size, end_threshold,
                                  min_trim_size, check_barcodes, forward_or_reverse)

    def find_end_trim(self, adapters, end_size, extra_trim_size, end_threshold,
                      scoring_scheme_vals, min_trim_size, check_barcodes, forward_or_reverse):
        window = self.seq[-end_size:]
        for adapter in adapters:
            if not adapter.end_sequence:
                continue
            hit = align_adapter(window, adapter.end_sequence[1], scoring_scheme_vals)
            self._apply_end_hit(adapter, hit, end_size, extra_trim_size, end_threshold,
                                min_trim_size, check_barcodes, forward_or_reverse)

    def find_middle_adapters(self, adapters, middle_threshold, extra_middle_trim_good_side,
                             extra_middle_trim_bad_side, scoring_scheme_vals,
                             start_sequence_names, end_sequence_names):
        """Whole-read scan, re-aligning the same adapter after masking each strong hit."""
        masked = self.get_seq_with_start_end_adapters_trimmed()
        for adapter_name, adapter_seq in adapters:
            while True:
                full, _, read_start, read_end = align_adapter(masked, adapter_seq, scoring_scheme_vals)
                if full < middle_threshold:
                    break
                masked = masked[:read_start] + '-' * (read_end - read_start) + masked[read_end:]
                self._apply_middle_hit(adapter_name, full, read_start, read_end,
                                       extra_middle_trim_good_side, extra_middle_trim_bad_side,
                                       start_sequence_names, end_sequence_names)

    # --- decision rules shared with the batched drivers -------------------------------------
    def _apply_start_hit(self, adapter, hit, end_size, extra_trim_size, end_threshold, min_trim_size,
                         check_barcodes, forward_or_reverse):
        full, partial, read_start, read_end = hit
        if partial > end_threshold and read_end != end_size and read_end - read_start >= min_trim_size:
            self.start_trim_amount = max(self.start_trim_amount, read_end + extra_trim_size)
            self.start_adapter_alignments.append((adapter, full, partial, read_start, read_end))
        if check_barcodes and adapter.is_barcode() and adapter.barcode_direction() == forward_or_reverse:
            self.start_barcode_scores[adapter.get_barcode_name()] = full

    def _apply_end_hit(self, adapter, hit, end_size, extra_trim_size, end_threshold, min_trim_size,
                       check_barcodes, forward_or_reverse):
        full, partial, read_start, read_end = hit
        if partial > end_threshold and read_start != 0 and read_end - read_start >= min_trim_size:
            self.end_trim_amount = max(self.end_trim_amount, (end_size - read_start) + extra_trim_size)
            self.end_adapter_alignments.append((adapter, full, partial, read_start, read_end))
        if check_barcodes and adapter.is_barcode() and adapter.barcode_direction() == forward_or_reverse:
            self.end_barcode_scores[adapter.get_barcode_name()] = full

    def _apply_middle_hit(self, adapter_name, full, read_start, read_end, good_side, bad_side,
                          start_sequence_names, end_sequence_names):
        self.middle_adapter_positions.update(range(read_start, read_end))
        self.middle_hit_str += '  %s (read coords: %d-%d, identity: %.1f%%)\n' % (
            adapter_name, read_start, read_end, full)
        trim_start = read_start - (bad_side if adapter_name in start_sequence_names else good_side)
        trim_end = read_end + (bad_side if adapter_name in end_sequence_names else good_side)
        self.middle_trim_positions.update(range(trim_start, trim_end))

    # --- verbose views (porechop_abi/nanopore_read.py:254-406) ----------------------------------
    # The drivers print these at verbosity 2 (formatted_start_and_end_seq, middle_adapter_results)
    # and 3 (full_start_end_output). Red = the trimmed adapter bases, yellow = the extra trim.
    def formatted_start_seq(self, end_size, extra_trim_size):
        window = self.seq[:end_size]
        if not self.start_trim_amount:
            return window
        n_red = self.start_trim_amount - extra_trim_size
        head = red(window[:n_red]) if n_red else ''
        return head + yellow(window[n_red:n_red + extra_trim_size]) + window[n_red + extra_trim_size:]

    def formatted_end_seq(self, end_size, extra_trim_size):
        window = self.seq[-end_size:]
        if not self.end_trim_amount:
            return window
        n_red = self.end_trim_amount - extra_trim_size
        tail = red(window[-n_red:]) if n_red else ''
        # slices as the reference takes them (n_red == 0 makes the yellow slice [-extra:0], empty)
        return window[:-(n_red + extra_trim_size)] + yellow(window[-(n_red + extra_trim_size):-n_red]) + tail

    def formatted_whole_seq(self, extra_trim_size):
        if not self.start_trim_amount and not self.end_trim_amount:
            return self.seq
        n_start = self.start_trim_amount - extra_trim_size if self.start_trim_amount else 0
        n_end = self.end_trim_amount - extra_trim_size if self.end_trim_amount else 0
        if n_start + n_end >= len(self.seq):
            return red(self.seq)
        head = red(self.seq[:n_start]) if self.start_trim_amount else ''
        tail = red(self.seq[-n_end:]) if self.end_trim_amount else ''
        mid = self.seq[n_start:len(self.seq) - n_end]
        if len(mid) <= 2 * extra_trim_size:
            mid = yellow(mid)
        else:
            if self.start_trim_amount:
                mid = yellow(mid[:extra_trim_size]) + mid[extra_trim_size:]
            if self.end_trim_amount:
                mid = mid[:-extra_trim_size] + yellow(mid[-extra_trim_size:])
        return head + mid + tail

    def formatted_start_and_end_seq(self, end_size, extra_trim_size, check_barcodes):
        out = ''
        if check_barcodes:
            out += 'start: %s (%.1f%%), end: %s (%.1f%%), barcode call: %s   ' % (
                self.best_start_barcode[0], self.best_start_barcode[1], self.best_end_barcode[0],
                self.best_end_barcode[1], self.barcode_call)
        if len(self.seq) <= 2 * end_size:
            return out + self.formatted_whole_seq(extra_trim_size)
        return out + self.formatted_start_seq(end_size, extra_trim_size) + '...' + \
            self.formatted_end_seq(end_size, extra_trim_size)

    @staticmethod
    def get_alignment_string(aln):
        """One recorded alignment (adapter, full, partial, read_start, read_end) as
        full_start_end_output lists it (nanopore_read.py:331-333)."""
        return '%s, full score=%s, partial score=%s, read position: %s-%s' % (
            aln[0].name, str(aln[1]), str(aln[2]), str(aln[3]), str(aln[4]))

    def full_start_end_output(self, end_size, extra_trim_size, check_barcodes):
        lines = [self.name, '  start: ' + self.formatted_start_seq(end_size, extra_trim_size) + '...']
        if self.start_adapter_alignments:
            lines.append('    start alignments:')
            lines += ['      ' + self.get_alignment_string(a) for a in self.start_adapter_alignments]
        lines.append('  end:   ...' + self.formatted_end_seq(end_size, extra_trim_size))
        if self.end_adapter_alignments:
            lines.append('    end alignments:')
            lines += ['      ' + self.get_alignment_string(a) for a in self.end_adapter_alignments]
        if check_barcodes:
            def listing(scores):
                return ', '.join('%s (%.1f%%)' % (k, v) for k, v in scores.items())
            lines += ['  Barcodes:',
                      '    start barcodes:        ' + listing(self.start_barcode_scores),
                      '    end barcodes:          ' + listing(self.end_barcode_scores),
                      '    best start barcode:    %s (%.1f%%)' % self.best_start_barcode,
                      '    best end barcode:      %s (%.1f%%)' % self.best_end_barcode]
            if self.albacore_barcode_call is not None:
                lines.append('    albacore barcode call: ' + self.albacore_barcode_call)
            lines.append('    final barcode call:    ' + self.barcode_call)
        return '\n'.join(lines) + '\n'

    def formatted_middle_seq(self):
        """The trimmed read around its middle hits (100 bases either side of the trim positions):
        adapter bases red, the extra middle trim yellow; None without middle hits."""
        if not self.middle_adapter_positions:
            return None
        seq = self.get_seq_with_start_end_adapters_trimmed()
        lo = max(0, min(self.middle_trim_positions) - 100)
        hi = min(len(seq), max(self.middle_trim_positions) + 100)
        out = [] if lo == 0 else ['(%d bp)...' % lo]
        last = None
        for i in range(lo, hi):
            c = RED if i in self.middle_adapter_positions else (YELLOW if i in self.middle_trim_positions else None)
            if c != last:
                out.append(END_FORMATTING + (c or ''))
                last = c
            out.append(seq[i])
        if last is not None:
            out.append(END_FORMATTING)
        if hi != len(seq):
            out.append('...(%d bp)' % (len(seq) - hi))
        return ''.join(out)

    def middle_adapter_results(self, verbosity):
        if not self.middle_adapter_positions:
            return ''
        out = self.name + '\n' + self.middle_hit_str
        if verbosity > 1:
            out += self.formatted_middle_seq() + '\n'
        return out

    def determine_barcode(self, barcode_threshold, barcode_diff, require_two_barcodes):
        """Barcode call from the start/end full-adapter identities (stable sorts: ties keep
        insertion order, i.e. adapter order, exactly like the reference)."""
        starts = sorted(self.start_barcode_scores.items(), reverse=True, key=lambda x: x[1])
        ends = sorted(self.end_barcode_scores.items(), reverse=True, key=lambda x: x[1])
        if starts:
            self.best_start_barcode = starts[0]
        if len(starts) > 1:
            self.second_best_start_barcode = starts[1]
        if ends:
            self.best_end_barcode = ends[0]
        if len(ends) > 1:
            self.second_best_end_barcode = ends[1]

        call = 'none'
        if require_two_barcodes:
            bs, be = self.best_start_barcode, self.best_end_barcode
            if (bs[1] >= barcode_threshold and be[1] >= barcode_threshold and
                    bs[1] >= self.second_best_start_barcode[1] + barcode_diff and
                    be[1] >= self.second_best_end_barcode[1] + barcode_diff and bs[0] == be[0]):
                call = bs[0]
        else:
            merged, seen = [], set()
            for name, score in sorted(starts + ends, reverse=True, key=lambda x: x[1]):
                if name not in seen:
                    merged.append((name, score))
                    seen.add(name)
            best = merged[0] if merged else ('none', 0.0)
            second = merged[1] if len(merged) > 1 else ('none', 0.0)
            if best[1] >= barcode_threshold and best[1] >= second[1] + barcode_diff:
                call = best[0]
        self.barcode_call = call
        if self.albacore_barcode_call is not None and self.barcode_call != self.albacore_barcode_call:
            self.barcode_call = 'none'


def parse_alignment_result(result_string):
    """The reference's parse of "rs,re,as,ae,score,pid1,pid2" (nanopore_read.py:485-500)."""
    parts = result_string.split(',')
    read_start = int(parts[0])
    if read_start == -1:
        return 0.0, 0.0, -1, 0
    return float(parts[6]), float(parts[5]), read_start, int(parts[1]) + 1


def align_adapter(read_seq, adapter_seq, scoring_scheme_vals):
    """(full_adapter_identity, aligned_region_identity, read_start, read_end_exclusive)."""
    return parse_alignment_result(adapter_alignment(read_seq, adapter_seq, scoring_scheme_vals))


def add_number_to_read_name(read_name, number):
    for sep in ('\t', ' '):
        if sep in read_name:
            return read_name.replace(sep, '_%d%s' % (number, sep), 1)
    return '%s_%d' % (read_name, number)
