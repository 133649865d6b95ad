/*
 * Job types the CPU engine may hold: those of processes outside the device subset and of instances
 * handed off to the engine.  JOB_BATCH:ACTIVATE of such a type stays with the engine
 * (JobBatchActivateProcessor.java:60-143 activates across every instance in JOB_ACTIVATABLE order,
 * and the adapter does not read the engine's rows).  Not compiled in this image (no JDK).
 */
package io.camunda.zeebe.zbhip;

import io.camunda.zeebe.engine.state.instance.JobRecordValue;
import io.camunda.zeebe.protocol.ZbColumnFamilies;
import java.nio.charset.StandardCharsets;
import java.util.HashSet;
import java.util.Set;
import java.util.regex.Matcher;
import java.util.regex.Pattern;
import org.agrona.concurrent.UnsafeBuffer;

final class JobTypes {
  static final int JOBS_COLUMN_FAMILY = ZbColumnFamilies.JOBS.ordinal();
  // zeebe:taskDefinition type="..." (static types; `=` expressions are refused by the compiler anyway)
  private static final Pattern TYPE = Pattern.compile("taskDefinition[^>]*?\\stype=\"([^\"=][^\"]*)\"");

  private JobTypes() {}

  static Set<String> of(final byte[] bpmnXml) {
    final Set<String> out = new HashSet<>();
    final Matcher m = TYPE.matcher(new String(bpmnXml, StandardCharsets.UTF_8));
    while (m.find()) {
      out.add(m.group(1));
    }
    return out;
  }

  // <message name="..."> (static names; the subset of the device's message catch events)
  private static final Pattern MESSAGE = Pattern.compile("<(?:\\w+:)?message\\b[^>]*?\\sname=\"([^\"=][^\"]*)\"");

  /** Static message names a BPMN XML declares (config 5: the PUBLISH commands the device takes). */
  static Set<String> messageNames(final byte[] bpmnXml) {
    final Set<String> out = new HashSet<>();
    final Matcher m = MESSAGE.matcher(new String(bpmnXml, StandardCharsets.UTF_8));
    while (m.find()) {
      out.add(m.group(1));
    }
    return out;
  }

  /** The job type of a JOBS column-family value (JobRecordValue, DbJobState.java:112-157). */
  static String typeOfJobsValue(final byte[] value) {
    final JobRecordValue v = new JobRecordValue();
    v.wrap(new UnsafeBuffer(value), 0, value.length);
    return v.getRecord().getType();
  }
}
